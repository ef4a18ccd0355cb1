"""CPU: the oracle (test infrastructure, oracle/inflate_oracle.c) under AddressSanitizer and
UndefinedBehaviorSanitizer ("Sanitizers: none").

oracle/san.mk builds oracle/_san/oracle_san (host gcc; no GPU code).  Every golden vector of
tests/golden/manifest.json is inflated from an exact-size heap copy (a read past the stream is an
ASan report), its result checked against the manifest (length + SHA-256, or an error where the
reference errs), and each stream is inflated again cut at 16 lengths and with 16 single-bit flips
(the error paths), all without a sanitizer report (-fno-sanitize-recover: any report aborts)."""
import hashlib
import json
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, GOLD)
from zgen import stream_of  # noqa: E402

MAN = json.load(open(os.path.join(GOLD, "manifest.json")))
VECS = [v for v in MAN["vectors"] if "stream" in v or "zgen" in v]


def _build():
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "-f", "san.mk"],
                       capture_output=True, text=True)
    if r.returncode != 0:
        if "asan" in r.stderr.lower() or "sanitize" in r.stderr.lower():
            pytest.skip("gcc without the sanitizer runtimes: " + r.stderr[-200:])
        raise AssertionError(r.stderr)
    return os.path.join(ROOT, "oracle", "_san", "oracle_san")


def test_oracle_under_asan_ubsan(tmp_path):
    exe = _build()
    jobs = []
    with open(tmp_path / "list.txt", "w") as lf:
        for i, v in enumerate(VECS):
            sp, op = tmp_path / f"s{i}.bin", tmp_path / f"o{i}.bin"
            sp.write_bytes(stream_of(v, GOLD))
            lf.write(f"{sp} {op} 0\n")
            jobs.append((v, op))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=99",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=98")
    r = subprocess.run([exe, str(tmp_path / "list.txt")], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    res = [tuple(int(x) for x in ln.split()) for ln in r.stdout.split("\n") if ln.strip()]
    assert len(res) == len(jobs)
    for (v, op), (rc, ln) in zip(jobs, res):
        if v.get("reference_reads_past_buffer") or not v["ref_ok"]:
            assert rc != 0, v["name"]
            continue
        assert rc == 0, v["name"]
        out = op.read_bytes()
        assert len(out) == v["out_len"] == ln and hashlib.sha256(out).hexdigest() == v["out_sha256"], v["name"]
