"""The drop-in boundary: include/timewarp.h vs the shipped library and the
ctypes mirror.  No device calls (CPU suite)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from timewarp import abi, isa
from timewarp.engine import EXPORTS, LIB_PATH, load_library

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "timewarp.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(tw_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    if not os.path.exists(LIB_PATH):
        pytest.skip("libtimewarp.so not built")
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (tw_\w+)", out))
    declared = _declared()
    assert declared, "no declarations parsed"
    missing = [s for s in declared if s not in exported]
    assert not missing, f"declared but not exported: {missing}"
    assert sorted(EXPORTS) == declared


def test_library_loads_without_device():
    if not os.path.exists(LIB_PATH):
        pytest.skip("libtimewarp.so not built")
    lib = load_library()
    assert b"gfx950" in lib.tw_version()
    assert lib.tw_strerror(-2) == b"no HIP device"
    # every status the header declares has its own message
    for name, val in re.findall(r"(TW_(?:OK|ERR_[A-Z_]+))\s*=\s*(-?\d+)", open(HEADER).read()):
        assert lib.tw_strerror(int(val)) != b"unknown error", name


def test_isa_mirror_in_sync():
    src = open(HEADER).read()
    for name, val in re.findall(r"TW_OP_([A-Z_]+)\s*=\s*(\d+)", src):
        assert getattr(isa, "OP_" + name) == int(val)


CHECK_C = r"""
#include <stdio.h>
#include <stddef.h>
#include "timewarp.h"
#define F(T, f) printf(#T "." #f " %zu\n", offsetof(T, f));
int main(void) {
  printf("tw_scenario_desc %zu\ntw_replica_result %zu\ntw_stats %zu\ntw_insn %zu\ntw_lp_state %zu\n"
         "tw_table_draw %zu\n",
         sizeof(tw_scenario_desc), sizeof(tw_replica_result), sizeof(tw_stats), sizeof(tw_insn),
         sizeof(tw_lp_state), sizeof(tw_table_draw));
  %FIELDS%
  return 0;
}
"""


def test_struct_layout_matches_ctypes(tmp_path):
    fields = []
    for T, cls in (("tw_scenario_desc", abi.TwScenarioDesc), ("tw_replica_result", abi.TwReplicaResult),
                   ("tw_stats", abi.TwStats), ("tw_lp_state", abi.TwLpState),
                   ("tw_table_draw", abi.TwTableDraw)):
        for f, _ in cls._fields_:
            fields.append(f"F({T}, {f})")
    src = tmp_path / "chk.c"
    src.write_text(CHECK_C.replace("%FIELDS%", "\n  ".join(fields)))
    exe = tmp_path / "chk"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split("\n") if line)
    assert int(got["tw_scenario_desc"]) == C.sizeof(abi.TwScenarioDesc)
    assert int(got["tw_replica_result"]) == C.sizeof(abi.TwReplicaResult)
    assert int(got["tw_stats"]) == C.sizeof(abi.TwStats)
    assert int(got["tw_insn"]) == 8
    assert int(got["tw_lp_state"]) == C.sizeof(abi.TwLpState)
    assert int(got["tw_table_draw"]) == C.sizeof(abi.TwTableDraw)
    for T, cls in (("tw_scenario_desc", abi.TwScenarioDesc), ("tw_replica_result", abi.TwReplicaResult),
                   ("tw_stats", abi.TwStats), ("tw_lp_state", abi.TwLpState),
                   ("tw_table_draw", abi.TwTableDraw)):
        for f, _ in cls._fields_:
            assert int(got[f"{T}.{f}"]) == getattr(cls, f).offset, (T, f)
