"""Metrics dashboard (reference: visual/UiServer.java + src/main/resources/web/index.html).

Same HTTP contract as the reference's NanoHTTPD server on :8888:
  GET/POST ``/?act=data``       body ``{"<series>": lastX, ...}`` -> points with x > lastX per series
  GET      ``/?act=list_graph`` -> list of series ids
  GET      ``/``                -> the dashboard page (polls act=data every second)
plus ``POST /plot`` (the ingest endpoint, replacing the reference's gRPC ``plot`` RPC on
uiPort; body = list of {id, x, y}).  ThreadingHTTPServer, so ingest never blocks a reader.
Like the reference the server listens on two ports -- the dashboard on ``-DuiHttpPort``
(8888, visual/UiServer.java:36) and the workers' ingest on ``-DuiPort`` (8990,
Context.java:81) -- both serving every route.
"""
from __future__ import annotations

import json
import threading
from typing import Optional
from collections import defaultdict
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlparse

_PAGE = """<!doctype html><html><head><meta charset="utf-8"><title>ps_amd metrics</title>
<script src="https://cdn.plot.ly/plotly-latest.min.js"></script></head><body>
<div id="graphs"></div><script>
var last = {};
function poll(){
  fetch('/?act=data', {method:'POST', body: JSON.stringify(last)}).then(r=>r.json()).then(d=>{
    for (const id in d){
      var pts = d[id]; if (!pts.length) continue;
      var el = document.getElementById('g_'+id);
      if (!el){ el=document.createElement('div'); el.id='g_'+id; document.getElementById('graphs').appendChild(el);
        Plotly.newPlot(el, [{x:[], y:[], mode:'lines', name:id}], {title:id}); }
      Plotly.extendTraces(el, {x:[pts.map(p=>p[0])], y:[pts.map(p=>p[1])]}, [0]);
      last[id] = pts[pts.length-1][0];
    }
  }).finally(()=>setTimeout(poll, 1000));
}
poll();
</script></body></html>"""


class UiServer:
    def __init__(self, host: str = "127.0.0.1", port: int = 8888, plot_port: Optional[int] = None):
        self.series = defaultdict(list)
        self.lock = threading.Lock()
        srv = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _json(self, obj, code=200):
                b = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(b)))
                self.end_headers()
                self.wfile.write(b)

            def _body(self):
                n = int(self.headers.get("Content-Length", "0") or 0)
                return self.rfile.read(n) if n else b""

            def _route(self, body: bytes):
                u = urlparse(self.path)
                act = parse_qs(u.query).get("act", [""])[0]
                if u.path == "/plot":
                    pts = json.loads(body or b"[]")
                    if isinstance(pts, dict):
                        pts = [pts]
                    with srv.lock:
                        for p in pts:
                            srv.series[str(p["id"])].append((float(p["x"]), float(p["y"])))
                    return self._json({"ok": len(pts)})
                if act == "data":
                    last = json.loads(body) if body else {}
                    out = {}
                    with srv.lock:
                        for k, pts in srv.series.items():
                            lx = last.get(k)
                            out[k] = [p for p in pts if lx is None or p[0] > float(lx)]
                    return self._json(out)
                if act == "list_graph":
                    with srv.lock:
                        return self._json(sorted(srv.series))
                b = _PAGE.encode()
                self.send_response(200)
                self.send_header("Content-Type", "text/html; charset=utf-8")
                self.send_header("Content-Length", str(len(b)))
                self.end_headers()
                self.wfile.write(b)

            def do_GET(self):
                self._route(b"")

            def do_POST(self):
                self._route(self._body())

        self.httpd = ThreadingHTTPServer((host, port), H)
        self.port = self.httpd.server_address[1]
        self._servers = [self.httpd]
        self.plot_port = None
        if plot_port is not None:  # the workers' ingest port (reference uiPort)
            ingest = ThreadingHTTPServer((host, plot_port), H)
            self.plot_port = ingest.server_address[1]
            self._servers.append(ingest)
        self.threads = [threading.Thread(target=s.serve_forever, daemon=True) for s in self._servers]

    def start(self) -> "UiServer":
        for t in self.threads:
            t.start()
        return self

    def stop(self) -> None:
        for s in self._servers:
            s.shutdown()
            s.server_close()


def main():  # pragma: no cover - CLI
    import argparse
    import time

    import sys

    from ..config import Config

    # reference flags: -DuiHost, -DuiHttpPort (dashboard), -DuiPort (ingest)
    cfg = Config.from_args([a for a in sys.argv[1:] if a.startswith("-D")])
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default=cfg.ui_host)
    ap.add_argument("--port", type=int, default=cfg.ui_http_port)
    ap.add_argument("--plot-port", type=int, default=cfg.ui_port)
    a, _ = ap.parse_known_args()
    s = UiServer(a.host, a.port, a.plot_port).start()
    print(f"ps_amd UI on http://{a.host}:{s.port}/ (ingest on :{s.plot_port})", flush=True)
    while True:
        time.sleep(3600)


if __name__ == "__main__":  # pragma: no cover
    main()
