"""The hand-counted `s_waitcnt vmcnt(N)` waits of the event kernels, checked
on a fresh compile (CPU only: hipcc cross-compiles gfx950).

The record prefetch and the far-run prefetch are LDS-DMA loads in inline asm,
which the compiler's wait-count pass does not model; the code that reads their
LDS staging proves they landed with a counted vmcnt(N) (engine_dev.hpp
Lane::fetch_rec, run_commit, the LP child staging).  tools/waitcnt_audit.py
walks every instantiation's control-flow graph and fails if some path reaches
such a wait after fewer than N vector-memory instructions since the load it
guards -- e.g. a compiler change that merged or dropped a store of the
fixed-shape store tail.  The victim headers a throwTo step stages at its pop
(Lane::stage_victims, stream `vic`) are checked the same way."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(ROOT, "tools")
sys.path.insert(0, TOOLS)

import waitcnt_audit  # noqa: E402


@pytest.fixture(scope="module")
def engine_asm(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("asm") / "engine.s")
    src = os.path.join(ROOT, "time-warp_amd", "csrc", "engine.hip")
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                        "-S", "-o", out, src], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    return out


def _audit(path, capsys):
    old = sys.argv
    sys.argv = ["waitcnt_audit.py", path]
    try:
        rc = waitcnt_audit.main()
    finally:
        sys.argv = old
    return rc, capsys.readouterr().out


def test_counted_waits_cover_their_loads(engine_asm, capsys):
    rc, out = _audit(engine_asm, capsys)
    assert rc == 0, out
    assert "kernels with a short counted wait: 0" in out
    # every replica and LP instantiation has its prefetch wait checked on some path
    lines = [l for l in out.splitlines() if "counted waits" in l]
    assert len(lines) >= 9 and all("vmcnt[" in l and "[]" not in l for l in lines), out


def test_audit_flags_a_short_wait(engine_asm, tmp_path, capsys):
    # the same code with the record prefetch's wait raised past the store tail:
    # vmcnt(12) no longer proves the prefetch landed
    s = open(engine_asm).read()
    assert "s_waitcnt vmcnt(9) ; tw:pf" in s
    bad = tmp_path / "short.s"
    bad.write_text(s.replace("s_waitcnt vmcnt(9) ; tw:pf", "s_waitcnt vmcnt(12) ; tw:pf"))
    rc, out = _audit(str(bad), capsys)
    assert rc == 1 and "SHORT" in out, out


def test_audit_flags_a_short_victim_wait(engine_asm, tmp_path, capsys):
    # throw_to's wait for the victim headers stage_victims loaded at the pop:
    # vmcnt(4) is proved by the record prefetch's four loads issued after them;
    # vmcnt(6) would not be
    s = open(engine_asm).read()
    assert "s_waitcnt vmcnt(4) ; tw:vic" in s
    bad = tmp_path / "short_vic.s"
    bad.write_text(s.replace("s_waitcnt vmcnt(4) ; tw:vic", "s_waitcnt vmcnt(6) ; tw:vic"))
    rc, out = _audit(str(bad), capsys)
    assert rc == 1 and "SHORT" in out, out
