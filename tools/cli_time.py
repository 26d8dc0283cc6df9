#!/usr/bin/env python3
"""Wall clock of the `ray` CLI on config 4 (diagnostic, GPU box): the bare
process (usage error: dynamic loading + static initialisation, no HIP), and
full renders with --stats, each as a fresh process."""
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-project_amd", "python"))
import scenes  # noqa: E402

RAY = os.path.join(REPO, "raytracing-project_amd", "bin", "ray")


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    for _ in range(3):
        t = time.perf_counter()
        r = subprocess.run([RAY], capture_output=True)
        print(f"bare process (rc {r.returncode}): {(time.perf_counter() - t) * 1e3:.1f} ms", flush=True)
    text, mode = scenes.config_json(cfg)
    with tempfile.TemporaryDirectory() as td:
        js = os.path.join(td, "s.json")
        open(js, "w").write(text)
        for _ in range(3):
            t = time.perf_counter()
            r = subprocess.run([RAY, js, os.path.join(td, "o.png")] + (["--paper"] if mode else []) +
                               ["--stats", "--threads", "16"], capture_output=True, text=True)
            wall = (time.perf_counter() - t) * 1e3
            lines = r.stdout.strip().splitlines()
            print(f"render rc {r.returncode}: {wall:.1f} ms  {lines[-2] if len(lines) > 1 else ''}  {lines[-1] if lines else r.stderr[-300:]}",
                  flush=True)


if __name__ == "__main__":
    main()
