"""AddressSanitizer + UndefinedBehaviorSanitizer over the host code
(SURVEY.md §5 "ASan/UBSan on the host CPU restatement"): the JSON parser and
schema loader, the IR, the device-table compiler, the PNG writer and the C
oracle, built from their sources with -fsanitize=address,undefined
(tools/sanitize/Makefile) and driven over every example, torture and deep
scene plus malformed JSON (tools/sanitize/host_check.cpp)."""
import json
import os
import shutil
import subprocess

import pytest

import scenes
from conftest import REPO

SAN_DIR = os.path.join(REPO, "tools", "sanitize")
BIN = os.path.join(REPO, "raytracing-project_amd", "build", "sanitize", "host_check")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_code_under_asan_ubsan(tmp_path):
    r = subprocess.run(["make", "-s"], cwd=SAN_DIR, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    files = []
    cases = {n: scenes.with_dpi(scenes.load_example(n), 8) for n in ("penguin", "pokeballs", "snorlax")}
    cases.update(scenes.torture_scenes(dpi=8))
    cases.update(scenes.deep_scenes(dpi=8))
    cases["cfg5"] = json.loads(scenes.config_json(5, dpi=8)[0])
    for name, d in cases.items():
        p = tmp_path / f"{name}.json"
        p.write_text(json.dumps(d))
        files.append(str(p))
    files.append(str(tmp_path / "missing.json"))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([BIN, str(tmp_path / "o.png")] + files, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-1000:], r.stderr[-3000:])
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
    assert r.stdout.count("ok ") == len(cases)
