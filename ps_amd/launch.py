"""Job launcher with whole-job restart (SURVEY §5.3 recovery; the reference has none -- a dead
worker or server hangs the BSP barrier forever, net/PServer.java:251-258).

    python -m ps_amd.launch --nproc 8 [--max-restarts 2] [--backend nccl|gloo] -- python app.py ...

Spawns ``nproc`` ranks on this node (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
MASTER_PORT, one process per GPU), each in its own session so a failed attempt can be torn
down by process group.  When any rank exits non-zero (killed, faulted, or aborted by the
heartbeat watchdog, utils/fault.py) every other rank of the attempt is terminated and the whole
job is started again -- same world size, a fresh rendezvous port, ``PS_AMD_RESTART=<attempt>``
-- and the apps resume from the last COMMITTED checkpoint of ``checkpoint_dir``
(utils/checkpoint.py).  Exit status: 0 when an attempt finishes cleanly, else the first failing
rank's status after the last allowed restart.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from typing import List


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_attempt(cmd: List[str], nproc: int, attempt: int, env_extra: dict, poll_s: float = 0.05) -> int:
    port = _free_port()
    procs = []
    for r in range(nproc):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PS_AMD_RESTART=str(attempt), **env_extra)
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
    rc = 0
    clean = False
    # ranks run in their own sessions (terminal SIGINT does not reach them): forward SIGTERM /
    # SIGINT to the launcher into a teardown of the attempt
    def _on_signal(signum, frame):
        raise KeyboardInterrupt(f"signal {signum}")

    old = {sg: signal.signal(sg, _on_signal) for sg in (signal.SIGTERM, signal.SIGINT)}
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                clean = True
                return 0
            time.sleep(poll_s)
    finally:
        for sg, h in old.items():
            signal.signal(sg, h)
        if not clean:  # a failed rank, or the launcher itself interrupted: no rank may outlive it
            for p in procs:  # tear the attempt down: every rank's own process group
                if p.poll() is None:
                    try:
                        os.killpg(p.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
            deadline = time.time() + 10
            for p in procs:
                try:
                    p.wait(max(0.1, deadline - time.time()))
                except subprocess.TimeoutExpired:
                    try:
                        os.killpg(p.pid, signal.SIGKILL)
                    except ProcessLookupError:
                        pass
                    p.wait()
    return rc


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--nproc", type=int, default=1)
    ap.add_argument("--max-restarts", type=int, default=0)
    ap.add_argument("--backend", default="", help="forwarded as PS_AMD_BACKEND (auto|nccl|gloo)")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    if not cmd:
        ap.error("missing command")
    extra = {"PS_AMD_BACKEND": a.backend} if a.backend else {}
    rc = 0
    for attempt in range(a.max_restarts + 1):
        rc = run_attempt(cmd, a.nproc, attempt, extra)
        if rc == 0:
            return 0
        sys.stderr.write(f"[ps_amd.launch] attempt {attempt} failed (exit {rc})"
                         + ("; restarting from the last checkpoint\n" if attempt < a.max_restarts else "\n"))
    return rc


if __name__ == "__main__":
    sys.exit(main())
