"""Sample every thread of another process from OUTSIDE it (no GIL, no ptrace): per 20 ms, each
thread's name, state, kernel wait channel and current syscall (number + first args), as JSON lines.
usage: proc_sampler.py PID OUT.jsonl [period_s]   (exits when PID does)"""
import json
import os
import sys
import time


def _rd(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except Exception:
        return "?"


def main():
    pid, out = int(sys.argv[1]), sys.argv[2]
    period = float(sys.argv[3]) if len(sys.argv) > 3 else 0.02
    with open(out, "w") as fo:
        while os.path.exists(f"/proc/{pid}"):
            t = time.time()
            rows = []
            try:
                tids = os.listdir(f"/proc/{pid}/task")
            except Exception:
                break
            for tid in tids:
                base = f"/proc/{pid}/task/{tid}"
                st = _rd(base + "/stat")
                state = st.rsplit(")", 1)[-1].split()[0] if ")" in st else "?"
                rows.append([int(tid), _rd(base + "/comm"), state, _rd(base + "/wchan"), _rd(base + "/syscall")[:60]])
            fo.write(json.dumps({"t": t, "th": rows}) + "\n")
            time.sleep(period)


if __name__ == "__main__":
    main()
