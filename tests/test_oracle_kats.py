"""Oracle pinned against the reference's own known answers.

* doc-comment examples of MonadTimed.hs / Timed.hs (exact timestamps; pop
  counts hand-derived in SURVEY.md Appendix D),
* test/Test/Control/TimeWarp/Timed/ExceptionSpec.hs checkpoint orders,
in both queue modes (canonical (t,seq) and the pqueue-1.3.1.1 transcription).
"""
import pytest

import progs
from timewarp import isa

MODES = [0, 1]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("kat", progs.KATS, ids=lambda f: f.__name__)
def test_doc_kat(oracle_mod, kat, mode):
    scn, exp = kat()
    r = oracle_mod.run(scn, mode=mode)
    assert r.result["status"] == isa.REP_DONE
    assert r.result["final_t"] == exp["final_t"]
    assert r.result["events"] == exp["events"]
    stamps = [v for (t, node, tag, v) in r.traces if tag == progs.TAG_TS]
    assert stamps == exp["stamps"]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("case", progs.EXCEPTION_SPEC, ids=lambda f: getattr(f, "__name__", "lambda"))
def test_exception_spec(oracle_mod, case, mode):
    scn, exp = case()
    r = oracle_mod.run(scn, mode=mode)
    cps = [v for (t, node, tag, v) in r.traces if tag == progs.TAG_CP]
    assert cps == exp["cps"], f"{scn.name}: checkpoints {cps}"
    assert r.result["main_exc"] == exp["main_exc"]
    assert r.result["status"] == isa.REP_DONE
    if "final_t" in exp:
        assert r.result["final_t"] == exp["final_t"]
    if "events" in exp:
        assert r.result["events"] == exp["events"]
    if "cp_times" in exp:
        assert [t for (t, node, tag, v) in r.traces if tag == progs.TAG_CP] == exp["cp_times"]


def test_fork_costs_one_microsecond(oracle_mod):
    """fork: parent resumes at now+1 (TimedT.hs:340); 2 pops (Appendix A.2)."""
    scn, exp = progs.kat_state_clone()
    r = oracle_mod.run(scn)
    assert r.result["final_t"] == 1_000_001 and r.result["events"] == 3
