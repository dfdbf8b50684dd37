"""Data pipeline (DataSet / FileSource sharding / native BatchReader) and observability
(metrics JSONL, UI server HTTP contract of visual/UiServer.java)."""
import json
import os
import time
import urllib.request

import numpy as np
import torch

from ps_amd.data.dataset import (DataSet, FileSource, LibsvmParser, MemorySource, MnistDataSet, NativeBatchDataSet,
                                 synthetic_ctr)
from ps_amd.obs import metrics
from ps_amd.obs.ui_server import UiServer


def _csv(tmp_path, n=25, d=3):
    p = tmp_path / "d.csv"
    p.write_text("\n".join(",".join([str(i % 10)] + [str(i * 10 + j) for j in range(d)]) for i in range(n)) + "\n")
    return str(p)


def test_filesource_sharding_disjoint(tmp_path):
    path = _csv(tmp_path)
    seen = []
    for off in range(3):
        s = FileSource(path, offset=off, step=3)
        lines = []
        while (line := s.read_line()) is not None:
            lines.append(line)
        seen.append(lines)
    assert sum(len(x) for x in seen) == 25 and not (set(seen[0]) & set(seen[1]))


def test_libsvm_parser_and_dataset():
    lines = [f"{i % 2} {i}:{0.5 * i} {i + 1}:1.0" for i in range(10)]

    class DS(DataSet):
        def parse_feature(self, rows):
            y = torch.tensor([r[0].value for r in rows])
            idx = torch.tensor([[f.idx for f in r[1:]] for r in rows])
            return {"Y": y, "I": idx}

    ds = DS(MemorySource(lines, 0, 1), LibsvmParser(), batch_size=4, threads=1)
    batches = list(ds)
    assert [len(b["Y"]) for b in batches] == [4, 4, 2]
    assert batches[0]["I"][1].tolist() == [1, 2]
    ds.reset()
    assert ds.has_next() and len(ds.next()["Y"]) == 4


def test_mnist_dataset(tmp_path):
    p = tmp_path / "m.csv"
    p.write_text("\n".join(",".join([str(i % 10)] + ["255"] * 784) for i in range(7)))
    ds = MnistDataSet(str(p), 3, threads=2)
    rows = sum(len(b["Y"]) for b in ds)
    assert rows == 7


def test_native_reader_formats(tmp_path):
    path = _csv(tmp_path, 25, 3)
    r = NativeBatchDataSet(path, "csv", 4, dims=3, threads=3, offset=0, step=1)
    total, xs = 0, []
    for b in r:
        total += len(b["Y"])
        xs.append(b["X"])
    assert total == 25 and torch.cat(xs).shape == (25, 3)
    lp = tmp_path / "l.svm"
    lp.write_text("1 3:0.5 7:1.5\n0 2:1\n")
    b = NativeBatchDataSet(str(lp), "libsvm", 8, fields=3, threads=1, offset=0, step=1).next()
    assert b["I"].tolist() == [[3, 7, -1], [2, -1, -1]] and b["V"][0, 1] == 1.5
    cp = tmp_path / "c.txt"
    cp.write_text("1|0.5,1.5|11,12,13\n0|2,3|21,22,23\n")
    b = NativeBatchDataSet(str(cp), "ctr", 8, dims=2, fields=3, threads=1, offset=0, step=1).next()
    assert b["E"].tolist() == [[11, 12, 13], [21, 22, 23]] and b["X"][1, 1] == 3.0
    # rank sharding: offset 1 of step 2 keeps odd lines
    b = NativeBatchDataSet(path, "csv", 100, dims=3, threads=1, offset=1, step=2).next()
    assert b["X"][:, 0].tolist() == [10.0 * i for i in range(1, 25, 2)]


def test_synthetic_ctr_deterministic():
    a, b = synthetic_ctr(64, seed=3, wide_k=4), synthetic_ctr(64, seed=3, wide_k=4)
    assert all(torch.equal(a[k], b[k]) for k in a) and a["E"].shape == (64, 23) and a["X"].shape == (64, 45)


def test_metrics_jsonl_and_ui_server(tmp_path, monkeypatch):
    monkeypatch.setenv("PS_AMD_METRICS_PATH", str(tmp_path / "m.jsonl"))
    srv = UiServer("127.0.0.1", 0).start()
    try:
        client = metrics.UiClient("127.0.0.1", srv.port)
        metrics.set_client(client)
        metrics.reset()
        for i in range(5):
            metrics.plot("loss", 1.0 / (i + 1), i)
        metrics.log_step(step=1, samples_per_s=123.0)
        client.flush()
        time.sleep(0.3)
        assert metrics.series("loss")[-1] == (4.0, 0.2)
        base = f"http://127.0.0.1:{srv.port}"
        names = json.loads(urllib.request.urlopen(base + "/?act=list_graph").read())
        assert names == ["loss"]
        req = urllib.request.Request(base + "/?act=data", data=json.dumps({"loss": 2}).encode())
        data = json.loads(urllib.request.urlopen(req).read())
        assert [p[0] for p in data["loss"]] == [3.0, 4.0]
        assert b"plotly" in urllib.request.urlopen(base + "/").read()
        lines = (tmp_path / "m.rank0.jsonl").read_text().strip().splitlines()
        assert len(lines) == 6 and json.loads(lines[-1])["kind"] == "step"
    finally:
        metrics.set_client(None)
        srv.stop()


def test_reference_ui_flags_route_and_gate_plots():
    """-DuiHost/-DuiPort build the worker's UI client (Context.java:81-82, UiClient.java:25-27);
    only replica 0 of a -DisMajor=1 worker reports (Context.java:94-100); the server listens on
    the dashboard port (-DuiHttpPort) and the ingest port (-DuiPort)."""
    import json
    import time
    import urllib.request

    from ps_amd import context as C
    from ps_amd.config import Config
    from ps_amd.obs import metrics
    from ps_amd.obs.ui_server import UiServer

    srv = UiServer("127.0.0.1", 0, plot_port=0).start()
    saved = C.ctx.cfg
    try:
        metrics.set_client(None)
        for major, name in ((1, "major_loss"), (0, "minor_loss")):
            C.ctx.init(Config.from_args(["-Dmode=dist", "-DuiHost=127.0.0.1", f"-DuiPort={srv.plot_port}",
                                         f"-DisMajor={major}"]))
            C.ctx.model_index = 0
            metrics.plot(name, 0.5, 1)
            C.ctx.model_index = 1  # replica 1 never reports
            metrics.plot(name + "_r1", 0.5, 1)
            C.ctx.model_index = 0
        for c in list(metrics._auto.values()):
            c.flush()
        deadline = time.time() + 5
        got = []
        while time.time() < deadline:  # dashboard port serves what arrived on the ingest port
            with urllib.request.urlopen(f"http://127.0.0.1:{srv.port}/?act=list_graph", timeout=2) as r:
                got = json.loads(r.read())
            if "major_loss" in got:
                break
            time.sleep(0.05)
        assert got == ["major_loss"], got
        # without UI flags no client is built at all
        C.ctx.init(Config.from_args(["-Dmode=dist"]))
        assert Config.from_args([]).ui_address() is None
        assert metrics._auto_client() is None or "PS_AMD_UI_ADDR" in __import__("os").environ
    finally:
        C.ctx.init(saved)
        srv.stop()
