#!/usr/bin/env python3
"""Trace-kernel time of a scene at recursion limits 1..N (GPU box; diagnostic):
where the recursion row's time goes, bounce by bounce.

Usage: python tools/rec_sweep.py [config=6] [max_rec=6]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-project_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tools"))

import ablate  # noqa: E402
import scenes  # noqa: E402


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    base = json.loads(scenes.config_json(cfg)[0])
    for rec in range(1, top + 1):
        s = dict(base, medium=dict(base["medium"], recursion=rec))
        ablate.run(f"recursion {rec}", s, reps=2)


if __name__ == "__main__":
    main()
