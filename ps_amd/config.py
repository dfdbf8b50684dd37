"""Typed configuration (reference: Context.init reading JVM ``-D`` properties,
context/Context.java:60-88, and the flags documented in README.md:72-96).

Sources, lowest to highest precedence: dataclass defaults -> ``PS_AMD_*`` environment
variables -> reference-style ``-Dkey=value`` / ``--key value`` command-line arguments.
Every reference flag name is accepted, including the README spellings the reference code
never actually read (Q18): ``isPs`` == ``ps``, ``isAsync`` == ``isPsAsync``,
``mode=standalone`` == anything but ``dist``.
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

_ALIASES = {
    # reference name (Context.java / README)  ->  field
    "mode": "mode",
    "nTermDump": "n_term_dump",
    "logRandom": "log_random",
    "thread": "thread",
    "ps": "ps",
    "isPs": "ps",
    "isPsAsync": "ps_async",
    "isAsync": "ps_async",
    "workerNum": "worker_num",
    "isMajor": "is_major",
    "psPort": "ps_port",
    "psHost": "ps_host",
    "psAddrs": "ps_addrs",
    "uiPort": "ui_port",
    "uiHost": "ui_host",
    "uiHttpPort": "ui_http_port",
    "train": "train",
    "test": "test",
    # new
    "consistency": "consistency",
    "staleness": "staleness",
    "backend": "backend",
    "bucketMb": "bucket_mb",
    "compress": "compress",
    "clipNorm": "clip_norm",
    "checkpointDir": "checkpoint_dir",
    "checkpointEvery": "checkpoint_every",
    "metricsPath": "metrics_path",
    "seed": "seed",
    "fault": "fault",
    "heartbeatS": "heartbeat_s",
}


def _to_bool(v) -> bool:
    if isinstance(v, bool):
        return v
    return str(v).strip().lower() in ("1", "true", "yes", "on")


@dataclass
class Config:
    mode: str = "stand"  # "dist" = distributed, anything else = standalone
    n_term_dump: int = 20
    log_random: int = 10
    thread: int = 1  # replicas per process (micro-batches accumulated per PS round)
    ps: bool = False  # this process is a dedicated parameter server (TCP topology)
    ps_async: bool = False  # reference async (ASP) mode
    worker_num: int = 1
    is_major: bool = True
    ps_port: int = 8890
    ps_host: str = "127.0.0.1"
    ps_addrs: str = "127.0.0.1:8890"
    ui_port: int = 8990
    ui_host: str = "127.0.0.1"
    ui_http_port: int = 8888
    train: str = ""
    test: str = ""
    consistency: str = "bsp"  # bsp | ssp | asp
    staleness: int = 0
    backend: str = "auto"  # auto | nccl | gloo | tcp
    bucket_mb: float = 25.0
    compress: str = ""  # "" | onebit
    compress_warmup: int = 0  # full-precision PS rounds before the 1-bit push
    clip_norm: float = 0.0
    checkpoint_dir: str = ""
    checkpoint_every: int = 0
    metrics_path: str = ""
    seed: int = 1234
    fault: str = ""  # e.g. "kill:rank=1:step=5", "delay_push:ms=50", "drop_push:p=0.01"
    heartbeat_s: float = 0.0

    # ----------------------------------------------------------------- derived
    @property
    def ps_addr_list(self) -> List[str]:
        return [a.strip() for a in self.ps_addrs.split(",") if a.strip()]

    @property
    def effective_consistency(self) -> str:
        if self.ps_async and self.consistency == "bsp":
            return "asp"
        return self.consistency

    def given(self, name: str) -> bool:
        """True if ``name`` was set explicitly (a -D flag, --flag or PS_AMD_* variable)."""
        return name in self.__dict__.get("_given", ())

    def ui_address(self) -> Optional[Tuple[str, int]]:
        """(uiHost, uiPort) of the metrics UI when the job was told about one (-DuiHost /
        -DuiPort, Context.java:81-82 -> visual/UiClient.java:25-27), else None."""
        if self.given("ui_port") or self.given("ui_host"):
            return self.ui_host, int(self.ui_port)
        return None

    def set(self, key: str, value) -> None:
        name = _ALIASES.get(key, key.replace("-", "_"))
        if name == "mode":
            value = "dist" if str(value) in ("dist", "distributed") else "stand"
        f = {f.name: f for f in dataclasses.fields(self)}.get(name)
        if f is None:
            raise KeyError(f"unknown config key {key!r}")
        t = f.type if isinstance(f.type, type) else {"int": int, "float": float, "bool": bool, "str": str}[f.type]
        setattr(self, name, _to_bool(value) if t is bool else t(value))
        self.__dict__.setdefault("_given", set()).add(name)

    # ----------------------------------------------------------------- sources
    @classmethod
    def from_env(cls, environ=None) -> "Config":
        env = os.environ if environ is None else environ
        c = cls()
        for f in dataclasses.fields(c):
            k = "PS_AMD_" + f.name.upper()
            if k in env:
                c.set(f.name, env[k])
        return c

    @classmethod
    def from_args(cls, argv: Optional[Sequence[str]] = None, base: Optional["Config"] = None) -> "Config":
        """Parse ``-Dkey=value`` (reference style) and ``--key value`` / ``--key=value``."""
        c = base or cls.from_env()
        argv = list(argv or [])
        i = 0
        while i < len(argv):
            a = argv[i]
            if a.startswith("-D") and "=" in a:
                k, v = a[2:].split("=", 1)
                c.set(k, v)
            elif a.startswith("--"):
                body = a[2:]
                if "=" in body:
                    k, v = body.split("=", 1)
                elif i + 1 < len(argv) and not argv[i + 1].startswith("-"):
                    k, v = body, argv[i + 1]
                    i += 1
                else:
                    k, v = body, "1"
                c.set(k, v)
            i += 1
        return c

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)
