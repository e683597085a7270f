"""Small MonadTimed programs restating the reference's doc examples (KATs) and
test/Test/Control/TimeWarp/Timed/{ExceptionSpec,MonadTimedSpec}.hs cases in
the lowering DSL.  Shared by the oracle tests (CPU) and the GPU tests."""
from __future__ import annotations

import numpy as np

from timewarp import isa
from timewarp.program import Program
from timewarp.scenario import Scenario, Topology
from timewarp.timeunits import after, at, for_, minute, ms, now, sec, till

TAG_TS = 100   # `timestamp` / checkpoint value in the traced register
TAG_CP = 101   # ExceptionSpec checkPoint n

ALL = isa.MASK_ALL
ASYNC = 1 << isa.EXC_THREAD_KILLED        # AsyncException
ARITH = 1 << isa.EXC_ARITH                # ArithException (Overflow)
TK = isa.EXC_THREAD_KILLED
OVERFLOW = isa.EXC_ARITH


def single(p: Program, name: str = "prog", n_replicas: int = 1, max_slots: int = 32,
           max_timeouts: int = 8) -> Scenario:
    img = p.finalize()
    topo = Topology.from_out_lists(1, [[]])
    return Scenario(name=name, image=img, topo=topo, n_replicas=n_replicas, main_pc=img.pc_of("main"),
                    main_node=0, max_slots=max_slots, queue_capacity=64, run_capacity=16,
                    max_timeouts=max_timeouts)


def cp(c, n: int, reg: int = 0):
    """checkPoint n (ExceptionSpec.hs:256-287)."""
    c.seti(reg, n).trace(TAG_CP, reg)


def stamp(c, reg: int = 0):
    """`timestamp` (MonadTimed.hs:189-191): trace virtualTime."""
    c.now(reg).trace(TAG_TS, reg)


# ------------------------------------------------------------ doc KATs
def kat_wait_for_for():
    """MonadTimed.hs:119-120: wait (for 1 sec) >> wait (for 5 sec) >> timestamp."""
    p = Program()
    c = p.function("main")
    c.wait(for_(1, sec)).wait(for_(5, sec))
    stamp(c)
    c.end()
    return single(p, "kat_wait_for_for"), dict(final_t=6_000_000, events=2, stamps=[6_000_000])


def kat_wait_for_till():
    """MonadTimed.hs:121-122: wait (for 1 sec) >> wait (till 5 sec)."""
    p = Program()
    c = p.function("main")
    c.wait(for_(1, sec)).wait(till(5, sec))
    stamp(c)
    c.end()
    return single(p, "kat_wait_for_till"), dict(final_t=5_000_000, events=2, stamps=[5_000_000])


def kat_accumulator():
    """MonadTimed.hs:123-124: wait (for 10 minute 34 sec 52 ms)."""
    p = Program()
    c = p.function("main")
    c.wait(for_(10, minute, 34, sec, 52, ms))
    stamp(c)
    c.end()
    return single(p, "kat_accumulator"), dict(final_t=634_052_000, events=1, stamps=[634_052_000])


def kat_one_mcs():
    """MonadTimed.hs:187-188: wait (for 1 mcs) >> timestamp."""
    p = Program()
    c = p.function("main")
    c.wait(for_(1))
    stamp(c)
    c.end()
    return single(p, "kat_one_mcs"), dict(final_t=1, events=1, stamps=[1])


def kat_invoke_now():
    """MonadTimed.hs:296-297: invoke now (timestamp "")."""
    p = Program()
    c = p.function("main")
    c.invoke(now)
    stamp(c)
    c.end()
    return single(p, "kat_invoke_now"), dict(final_t=0, events=1, stamps=[0])


def kat_start_timer():
    """MonadTimed.hs:304-314: wait 10 s; timer <- startTimer; wait 5 ms; timer -> 5000."""
    p = Program()
    c = p.function("main")
    c.wait(for_(10, sec)).now(1)            # startTimer
    c.wait(for_(5, ms)).now(0).sub(0, 1)    # passedTime <- timer
    c.trace(TAG_TS, 0).end()
    return single(p, "kat_start_timer"), dict(final_t=10_005_000, events=2, stamps=[5_000])


def kat_schedule():
    """MonadTimed.hs:155-161: wait 10 s; schedule (after 3 s) p13; schedule (at 15 s) p15; p_now."""
    p = Program()
    c = p.function("main")
    c.wait(for_(10, sec))
    c.schedule(after(3, sec), "p")
    c.schedule(at(15, sec), "p")
    stamp(c)
    c.end()
    c = p.function("p")
    stamp(c)
    c.end()
    return single(p, "kat_schedule"), dict(final_t=15_000_000, events=7,
                                            stamps=[10_000_002, 13_000_000, 15_000_000])


def kat_invoke():
    """MonadTimed.hs:174-181: wait 10 s; invoke (after 3 s) p; invoke (after 3 s) p; invoke (at 20 s) p; p."""
    p = Program()
    c = p.function("main")
    c.wait(for_(10, sec))
    c.invoke(after(3, sec))
    stamp(c)
    c.invoke(after(3, sec))
    stamp(c)
    c.invoke(at(20, sec))
    stamp(c)
    stamp(c)
    c.end()
    return single(p, "kat_invoke"), dict(final_t=20_000_000, events=4,
                                          stamps=[13_000_000, 16_000_000, 20_000_000, 20_000_000])


def kat_timed_module():
    """Timed.hs:16-38: schedule (at 10 minute) hello; wait (for 9 minute); print."""
    p = Program()
    c = p.function("main")
    c.schedule(at(10, minute), "hello")
    c.wait(for_(9, minute))
    stamp(c)
    c.end()
    c = p.function("hello")
    stamp(c)
    c.end()
    return single(p, "kat_timed_module"), dict(final_t=600_000_000, events=4,
                                                stamps=[540_000_001, 600_000_000])


def kat_state_clone():
    """MonadTimed.hs:92-101: put 1; fork (put 10); wait (for 1 sec); print =<< get  -> 1
    (thread-local state is cloned on fork: registers are copied)."""
    p = Program()
    c = p.function("main")
    c.seti(0, 1)
    c.fork_("child")
    c.wait(for_(1, sec))
    c.trace(TAG_TS, 0).end()
    c = p.function("child")
    c.seti(0, 10).end()
    return single(p, "kat_state_clone"), dict(final_t=1_000_001, events=3, stamps=[1])


KATS = [kat_wait_for_for, kat_wait_for_till, kat_accumulator, kat_one_mcs, kat_invoke_now, kat_start_timer,
        kat_schedule, kat_invoke, kat_timed_module, kat_state_clone]


# --------------------------------------------------- ExceptionSpec cases
def exc_caught():
    """ExceptionSpec.hs:102-109: (throwM ThreadKilled >> cp -1) `catchAll` (cp 1)."""
    p = Program()
    c = p.function("main")
    h, done = c.label(), c.label()
    c.catch_(ALL, h)
    c.throw(TK)
    cp(c, -1)
    c.uncatch().jmp(done)
    c.bind(h)
    cp(c, 1)
    c.bind(done)
    c.end()
    return single(p, "exc_caught"), dict(cps=[1], main_exc=0)


def exc_caught_outside():
    """ExceptionSpec.hs:111-121: runEmu (wait 1 s >> throwM ThreadKilled) escapes runTimedT."""
    p = Program()
    c = p.function("main")
    c.wait(for_(1, sec)).throw(TK)
    cp(c, -1)
    c.end()
    return single(p, "exc_caught_outside"), dict(cps=[], main_exc=TK, final_t=1_000_000)


def exc_caught_outside_no_wait():
    """ExceptionSpec.hs:123-133: runEmu (throwM ThreadKilled) escapes runTimedT."""
    p = Program()
    c = p.function("main")
    c.throw(TK)
    cp(c, -1)
    c.end()
    return single(p, "exc_caught_outside_no_wait"), dict(cps=[], main_exc=TK, final_t=0, events=0)


def exc_wait_throw():
    """ExceptionSpec.hs:135-146: (wait 1 s >> throwM TK) `catchAll` cp 1; cp 2."""
    p = Program()
    c = p.function("main")
    h, done = c.label(), c.label()
    c.catch_(ALL, h)
    c.wait(for_(1, sec)).throw(TK)
    c.uncatch().jmp(done)
    c.bind(h)
    cp(c, 1)
    c.bind(done)
    cp(c, 2)
    c.end()
    return single(p, "exc_wait_throw"), dict(cps=[1, 2], main_exc=0)


def exc_wait_throw_forked():
    """ExceptionSpec.hs:148-159: fork_ (act `catchAll` cp 1); invoke (after 1 s) cp 2."""
    p = Program()
    c = p.function("main")
    c.fork_("child")
    c.invoke(after(1, sec))
    cp(c, 2)
    c.end()
    c = p.function("child")
    h = c.label()
    c.catch_(ALL, h)
    c.wait(for_(1, sec)).throw(TK)
    c.uncatch().end()
    c.bind(h)
    cp(c, 1)
    c.end()
    return single(p, "exc_wait_throw_forked"), dict(cps=[1, 2], main_exc=0,
                                                     cp_times=[1_000_000, 1_000_001])


def exc_catch_order():
    """ExceptionSpec.hs:161-171: throwM TK `catchAll` cp 1 `catchAll` cp -1; cp 2."""
    p = Program()
    c = p.function("main")
    h1, h2, done = c.label(), c.label(), c.label()
    c.catch_(ALL, h2)
    c.catch_(ALL, h1)
    c.throw(TK)
    c.uncatch().uncatch().jmp(done)
    c.bind(h1)
    cp(c, 1)
    c.uncatch().jmp(done)
    c.bind(h2)
    cp(c, -1)
    c.bind(done)
    cp(c, 2)
    c.end()
    return single(p, "exc_catch_order"), dict(cps=[1, 2], main_exc=0)


def exc_catch_scope(with_wait: bool):
    """ExceptionSpec.hs:173-193: a finished catch does not handle later exceptions."""
    p = Program()
    c = p.function("main")
    h_in, h_out, after_in, done = c.label(), c.label(), c.label(), c.label()
    c.catch_(ALL, h_out)
    c.catch_(ALL, h_in)
    cp(c, 1)
    if with_wait:
        c.wait(for_(1, sec))
    c.uncatch().jmp(after_in)
    c.bind(h_in)
    cp(c, -1)
    c.bind(after_in)
    if with_wait:
        c.wait(for_(1, sec))
    c.throw(TK)
    c.uncatch().jmp(done)
    c.bind(h_out)
    cp(c, 2)
    c.bind(done)
    cp(c, 3)
    c.end()
    return single(p, f"exc_catch_scope{'_wait' if with_wait else ''}"), dict(cps=[1, 2, 3], main_exc=0)


def exc_diff_catch(inner: bool):
    """ExceptionSpec.hs:195-217: typed handlers pick the matching layer."""
    p = Program()
    c = p.function("main")
    h_async, h_arith, done = c.label(), c.label(), c.label()
    c.catch_(ARITH, h_arith)   # outer: ArithException
    c.catch_(ASYNC, h_async)   # inner: AsyncException
    c.throw(TK if inner else OVERFLOW)
    c.uncatch().uncatch().jmp(done)
    c.bind(h_async)
    cp(c, 1 if inner else -1)
    c.uncatch().jmp(done)
    c.bind(h_arith)
    cp(c, -1 if inner else 1)
    c.bind(done)
    cp(c, 2)
    c.end()
    return single(p, f"exc_diff_catch_{'inner' if inner else 'outer'}"), dict(cps=[1, 2], main_exc=0)


def exc_handler_throw():
    """ExceptionSpec.hs:219-229: the inner handler rethrows Overflow, caught outside."""
    p = Program()
    c = p.function("main")
    h1, h2, done = c.label(), c.label(), c.label()
    c.catch_(ARITH, h2)
    c.catch_(ALL, h1)
    c.throw(TK)
    c.uncatch().uncatch().jmp(done)
    c.bind(h1)
    c.throw(OVERFLOW)
    c.bind(h2)
    cp(c, 1)
    c.bind(done)
    cp(c, 2)
    c.end()
    return single(p, "exc_handler_throw"), dict(cps=[1, 2], main_exc=0)


def exc_throw_to_correct():
    """ExceptionSpec.hs:231-242: tid <- fork (catch (wait 1 s) (Arith -> cp 1));
    throwTo tid Overflow; wait 2 s; cp 2."""
    p = Program()
    c = p.function("main")
    c.fork("child", ref=1)
    c.throw_to(1, OVERFLOW)
    c.wait(for_(2, sec))
    cp(c, 2)
    c.end()
    c = p.function("child")
    h = c.label()
    c.catch_(ARITH, h)
    c.wait(for_(1, sec))
    c.uncatch().end()
    c.bind(h)
    cp(c, 1)
    c.end()
    return single(p, "exc_throw_to_correct"), dict(cps=[1, 2], main_exc=0, cp_times=[1, 2_000_001])


def exc_throw_to_kill():
    """ExceptionSpec.hs:244-251: tid <- fork (wait 1 s >> cp -1); throwTo tid Overflow."""
    p = Program()
    c = p.function("main")
    c.fork("child", ref=1)
    c.throw_to(1, OVERFLOW)
    c.end()
    c = p.function("child")
    c.wait(for_(1, sec))
    cp(c, -1)
    c.end()
    return single(p, "exc_throw_to_kill"), dict(cps=[], main_exc=0, final_t=1)


EXCEPTION_SPEC = [exc_caught, exc_caught_outside, exc_caught_outside_no_wait, exc_wait_throw,
                  exc_wait_throw_forked, exc_catch_order, lambda: exc_catch_scope(False),
                  lambda: exc_catch_scope(True), lambda: exc_diff_catch(True), lambda: exc_diff_catch(False),
                  exc_handler_throw, exc_throw_to_correct, exc_throw_to_kill]


# ------------------------------------------------------ edge behaviours
def timeout_prog(tout: int, wt: int):
    """MonadTimedSpec.hs:275-286: timeout tout (wait wt; return (wt <= tout))
    `catch` (\\_ -> return (tout <= wt)).  Traces 1 = normal, 2 = timed out."""
    p = Program()
    c = p.function("main")
    h, done = c.label(), c.label()
    c.catch_(ALL, h)
    c.timeout_begin(tout, epoch_reg=3)
    c.wait(for_(wt))
    c.timeout_end()
    c.uncatch()
    c.seti(0, 1).trace(TAG_TS, 0).jmp(done)
    c.bind(h)
    c.seti(0, 2).trace(TAG_TS, 0)
    c.bind(done)
    c.end()
    return single(p, "timeout")


def kill_thread_prog(m_time: int, f1: int, f2: int):
    """MonadTimedSpec.hs:246-273: the grandchild cannot be killed; result var in node var 0."""
    p = Program()
    c = p.function("main")
    c.fork("child", ref=1)
    c.wait(for_(m_time))
    c.kill_thread(1)
    c.wait(for_(f1)).wait(for_(f2))
    c.nload(0, 0).trace(TAG_TS, 0).end()
    c = p.function("child")
    c.fork_("grandchild")
    c.wait(for_(f2))
    c.seti(0, 2).nstore(0, 0).end()
    c = p.function("grandchild")
    c.wait(for_(f1))
    c.seti(0, 1).nstore(0, 0).end()
    return single(p, "kill_thread")


def work_prog(life: int, period: int):
    """`work (for life) act` (MonadTimed.hs:201-202) with a ticking act: the act
    is killThread-ed at +life; ticks traced."""
    p = Program()
    c = p.function("main")
    c.work(for_(life), "ticker", ref=2)
    c.end()
    c = p.function("ticker")
    top = c.here()
    c.wait(for_(period))
    stamp(c)
    c.jmp(top)
    return single(p, "work")


def random_program(seed: int, n_threads: int = 6, n_replicas: int = 1):
    """Random fork/wait/throwTo/catch/timeout soup for differential GPU-vs-oracle tests."""
    rng = np.random.default_rng(seed)
    p = Program()
    names = [f"t{i}" for i in range(n_threads)]
    c = p.function("main")
    for i in range(1, n_threads):
        c.fork(names[i], ref=1)
        c.nstore(1, i % 4)
        c.wait(for_(int(rng.integers(0, 5))))
    c.jmp(names[0])
    for i, nm in enumerate(names):
        c = p.function(nm)
        h = c.label()
        c.catch_(ALL if rng.random() < 0.5 else ASYNC | ARITH, h)
        loop = c.here()
        for _ in range(int(rng.integers(2, 6))):
            r = rng.random()
            if r < 0.4:
                c.wait(for_(int(rng.choice([0, 1, 2, 3, 1000]))))
            elif r < 0.55:
                c.nload(1, int(rng.integers(0, 4))).throw_to(1, int(rng.choice([TK, OVERFLOW, 5])), 0)
            elif r < 0.7:
                stamp(c)
            elif r < 0.8:
                c.schedule(after(int(rng.integers(0, 4))), nm if rng.random() < 0.2 else names[-1])
            elif r < 0.9:
                c.timeout_begin(int(rng.integers(0, 6)), epoch_reg=3)
                c.wait(for_(int(rng.integers(0, 6))))
                c.timeout_end()
            else:
                c.addi(0, 1)
        c.addi(0, 1).seti(2, int(rng.integers(1, 4)))
        c.jlt(0, 2, loop)
        c.uncatch().end()
        c.bind(h)
        c.trace(TAG_CP, 3)
        c.end()
    s = single(p, f"random{seed}", n_replicas=n_replicas, max_slots=256, max_timeouts=4096)
    s.queue_capacity = 4096
    s.run_capacity = 512
    return s


# ------------------------------------------- handler stack, payloads (ABI 2)
def deep_catch_prog(depth: int, max_frames: int = 8, payload: int = 0):
    """A handler stack `depth` frames deep (TimedT's `_handlers` list grows per
    `catch`, TimedT.hs:84,198): catch frames alternate Arith / async masks, a
    `timeout` finally frame sits at every third level.  A forked child is
    thrown a ThreadKilled carrying `payload` (throwTo, TimedT.hs:357-368) while
    parked under its whole stack; each handler traces its level and the value,
    then throws Overflow, which unwinds to the next Arith frame below
    (ExceptionSpec.hs:219-229 chained).  Checkpoints: the levels caught."""
    p = Program()
    c = p.function("main")
    c.seti(0, payload) if -(1 << 31) <= payload < (1 << 31) else c.seti(0, payload)
    c.fork("child", ref=1)
    c.wait(for_(5))
    c.throw_to(1, TK, 0)
    c.wait(for_(100))
    c.end()
    c = p.function("child")
    hs = [c.label() for _ in range(depth)]
    for i in range(depth):
        if i % 3 == 2:
            c.timeout_begin(1_000_000, epoch_reg=3)   # finally frame (watchdog far away)
        else:
            c.catch_(ARITH if i % 2 == 0 else ASYNC, hs[i])
    c.wait(for_(1000))                                # parked under the whole stack
    cp(c, -1)
    c.end()
    for i in range(depth):
        c.bind(hs[i])
        c.seti(2, i).trace(TAG_CP, 2)                  # level that caught it
        c.trace(TAG_TS, 0)                             # the exception value (r0)
        c.throw(OVERFLOW)                              # unwinds to the next Arith frame below
    s = single(p, f"deep_catch_{depth}", max_slots=32, max_timeouts=64)
    s.max_frames = max_frames
    return s


def payload_prog(value: int):
    """`data SignalException = ValueReceived Int` (examples/token-ring/Main.hs:156)
    thrown with a full-width Int: the handler traces the value it received."""
    p = Program()
    c = p.function("main")
    c.fork("child", ref=1)
    c.seti(0, value)
    c.throw_to(1, isa.EXC_USER0, 0)
    c.end()
    c = p.function("child")
    h = c.label()
    c.catch_(1 << isa.EXC_USER0, h)
    c.wait(for_(10))
    c.uncatch().end()
    c.bind(h)
    c.trace(TAG_TS, 0)
    c.end()
    return single(p, f"payload_{value}")
