"""Lowering of MonadTimed / MonadDialog scenarios to thread programs.

A scenario of the reference is Haskell code polymorphic in ``m`` under
``MonadTimed``/``MonadDialog`` constraints (e.g. ``WorkMode``,
examples/token-ring/Main.hs:93-98).  Here the same scenario is written as
per-node handler state machines against a small assembler whose methods keep
the reference's names and meaning:

===============================  ==============================================
reference (file:line)            lowering
===============================  ==============================================
``wait (for t)`` / ``till``      ``Code.wait(for_(t))`` -> WAIT_REL / WAIT_ABS
  (MonadTimed.hs:125, TimedT.hs:343-355)
``fork act`` (TimedT.hs:326-342) ``Code.fork(entry, ref=r)`` -> FORK (+1 µs)
``fork_``  (MonadTimed.hs:194)   ``Code.fork_(entry)``
``schedule t act`` (:162-163)    ``Code.schedule(t, entry)`` = fork_ of a stub
                                 ``wait t; jmp entry``
``invoke t act`` (:182-183)      ``Code.invoke(t)`` = wait
``work t act`` (:201-202)        ``Code.work(t, entry)``
``killThread`` (:205-206)        ``Code.kill_thread(ref)``
``throwTo`` (TimedT.hs:357-368)  ``Code.throw_to(ref, exc, val)``
``throwM`` / ``catch``           ``Code.throw`` / ``Code.catch_(mask, handler)``
``timeout t act`` (:370-376)     ``Code.timeout_begin(t)`` ... ``timeout_end()``
``virtualTime`` / ``myThreadId`` ``Code.now(r)`` / ``Code.my_thread_id(r)``
``send addr msg`` (MonadDialog.hs:154-156)  ``Code.send(link, kind, payload)``
``listen (AtPort p) [..]`` (:204-211)       ``Code.listen(set)``
``listenR binding ls raw`` (:226-256)       ``Code.listen(set)`` with
                                 ``listener_set(..., raw=fn)``
``reply`` (:177-180)             ``Code.reply_link(r, r_in)`` + ``send``
``userStateR`` (socket-state :91-93)  ``Code.user_state_load/_store`` (a state
                                 cell per incoming link)
``close`` / ``closeR``           ``Code.close_conn`` (the link's state cell is
  (MonadTransfer.hs:139-142,162)  reset: the next connection starts fresh)
===============================  ==============================================

Registers r0..r3 are per-thread int64 and are copied into forked children
(the closure a forked action captures).  A thread ref (``fork``'s result) is an
opaque register value usable only by throw_to / kill_thread.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Union

import numpy as np

from . import isa
from .timeunits import TimeSpec


class Label:
    __slots__ = ("name", "pc")

    def __init__(self, name: str):
        self.name = name
        self.pc: Optional[int] = None

    def __repr__(self):
        return f"Label({self.name}@{self.pc})"


Imm = Union[int, Label]


def _enc(op: int, a: int = 0, b: int = 0) -> int:
    return (op & 0xFF) | ((a & 0xFF) << 8) | ((b & 0xFFFF) << 16)


_ALU_B_FREE = (isa.OP_SETI, isa.OP_SETK, isa.OP_ADDI, isa.OP_MULI, isa.OP_NOW, isa.OP_NODE)


def _fuse_pairs(insns: np.ndarray) -> None:
    """Peephole over the resolved image: an instruction pair becomes one
    instruction in the pair's first slot (include/timewarp.h):

      LINK a,k ; SEND a,..    -> SEND with TW_SEND_VIA_LINK (imm = k)
      RLINK a,r ; SEND a,..   -> SEND with TW_SEND_VIA_RLINK (r in b bits 12-13)
      op a,.. ; NSTORE a,v    -> op with TW_ALU_NSTORE | v  (op: SETI SETK ADDI
                                 MULI NOW NODE, whose b is otherwise unused)
      TRACE a,t ; TRACE a2,t2 -> TRACE with TW_TRACE_PAIR | a2 << 13 | t2 (t2 < 8192)

    The fused instruction continues at pc + 2.  The pair's second instruction
    stays where it is, so a jump to it still runs it alone; pcs, yields and
    trace terms are those of the unfused image (one instruction, one
    interpreter pass and one step count fewer per pair).  A SEND pair whose
    payload register is `a` is left alone (the payload would be the link the
    fused half just computed).  Every rewrite reads the original image, so
    overlapping pairs (three TRACEs in a row) fuse consistently."""
    orig = insns.copy()
    for i in range(len(orig) - 1):
        w, w2 = int(orig[i, 0]), int(orig[i + 1, 0])
        op, op2 = w & 0xFF, w2 & 0xFF
        a, a2, b, b2 = (w >> 8) & 0xFF, (w2 >> 8) & 0xFF, w >> 16, w2 >> 16
        if op2 == isa.OP_SEND and op in (isa.OP_LINK, isa.OP_RLINK):
            if a != a2 or (b2 >> 10) != 0 or ((b2 >> 8) & 3) == (a & 3):
                continue
            if op == isa.OP_LINK:
                insns[i, 0] = _enc(isa.OP_SEND, a, b2 | isa.SEND_VIA_LINK)  # imm: LINK's k
            else:
                insns[i, 0] = _enc(isa.OP_SEND, a, b2 | isa.SEND_VIA_RLINK | ((b & 3) << 12))
                insns[i, 1] = 0
        elif op2 == isa.OP_NSTORE and op in _ALU_B_FREE and b == 0 and (a & 3) == (a2 & 3):
            insns[i, 0] = _enc(op, a, isa.ALU_NSTORE | (b2 & 3))
        elif op == isa.OP_TRACE and op2 == isa.OP_TRACE and b == 0 and 0 <= int(orig[i + 1, 1]) < 0x2000:
            insns[i, 0] = _enc(op, a, isa.TRACE_PAIR | ((a2 & 3) << 13) | int(orig[i + 1, 1]))


class Program:
    """Program image: insns + constant pool + listener sets + message kinds."""

    def __init__(self):
        self._insns: List[list] = []
        self.consts: List[int] = []
        self._cidx: Dict[int, int] = {}
        self._labels: Dict[str, Label] = {}
        self._deferred: List[Callable[[], None]] = []
        self.msg_kinds: Dict[str, int] = {}
        self.listener_sets: List[Dict[int, Label]] = []
        self.listener_inline: List[set] = []
        self.listener_raw: List[Optional[Callable[["Code", Label], None]]] = []
        self._nfresh = 0
        # fixed stubs (include/timewarp.h TW_PC_*): deliverer and timeout watchdog
        self._emit(isa.OP_WAIT_REG, 2)
        self._emit(isa.OP_DELIVER)
        self._emit(isa.OP_END)
        self._emit(isa.OP_WAIT_REG, 2)
        self._emit(isa.OP_TMO_FIRE)
        self._emit(isa.OP_END)
        assert self.pc == isa.PC_USER

    # ---------------------------------------------------------------- basics
    @property
    def pc(self) -> int:
        return len(self._insns)

    def _emit(self, op: int, a: int = 0, b: int = 0, imm: Imm = 0) -> None:
        self._insns.append([_enc(op, a, b), imm])

    def const(self, v: int) -> int:
        v = int(v)
        if v not in self._cidx:
            self._cidx[v] = len(self.consts)
            self.consts.append(v)
        return self._cidx[v]

    def label(self, name: Optional[str] = None) -> Label:
        if name is None:
            self._nfresh += 1
            name = f"_L{self._nfresh}"
        if name in self._labels:
            return self._labels[name]
        lab = Label(name)
        self._labels[name] = lab
        return lab

    def bind(self, lab: Label) -> Label:
        if lab.pc is not None:
            raise ValueError(f"label {lab.name} bound twice")
        lab.pc = self.pc
        return lab

    def function(self, name: str) -> "Code":
        """Start a code block at a (new or forward-declared) label."""
        self.bind(self.label(name))
        return Code(self)

    def kind(self, name: str) -> int:
        """Message kind id (the reference dispatches by message name, MonadDialog.hs:240)."""
        if name not in self.msg_kinds:
            self.msg_kinds[name] = len(self.msg_kinds)
        return self.msg_kinds[name]

    def listener_set(self, listeners: Dict[str, Union[str, Label]], inline: Sequence[str] = (),
                     raw: Optional[Callable[["Code", Label], None]] = None) -> int:
        """A `listen` binding's listener list: message name -> handler entry.

        `inline` names the messages whose handler runs in place in the
        delivering thread (ForkStrategy `const id`, MonadDialog.hs:114-117);
        the others are forked with `fork_` (the default, MonadDialog.hs:317).

        `raw` makes the binding a ``listenR`` (MonadDialog.hs:226-256): the raw
        listener runs first, in the handler's thread, for every message that
        reaches the port -- also for names without a typed listener
        (:240-244).  ``raw(code, accept)`` emits its body: jumping to
        ``accept`` is ``return True`` (the typed listener, if any, runs next,
        :246-253), ending the thread is ``return False``; an uncaught exception
        also ends the thread, which is what ``invokeRawListenerSafe``'s
        ``return False`` amounts to (:262-264).  The body sees the handler
        registers (r0 payload, r1 incoming link, r3 kind) and must leave r0
        and r1 as it found them; r2 and r3 are scratch (r3 is restored before
        the typed listener).  It is expanded once per message kind at
        `finalize`, since the ISA has no call/return."""
        unknown = set(inline) - set(listeners)
        if unknown and raw is None:
            raise ValueError(f"inline strategy for messages without a listener: {sorted(unknown)}")
        s = {self.kind(k): (v if isinstance(v, Label) else self.label(v)) for k, v in listeners.items()}
        self.listener_sets.append(s)
        self.listener_inline.append({self.kind(k) for k in inline})
        self.listener_raw.append(raw)
        return len(self.listener_sets) - 1

    def _expand_raw_listeners(self) -> None:
        """listenR: per (set, kind), an entry that runs the raw listener and
        continues to the typed listener (or ends) on `accept`.  Every set gets
        an entry for every message kind; `undeliverable` then means that no
        listener is bound at the destination port."""
        kinds = sorted(self.msg_kinds.values())
        no_listener: Optional[Label] = None
        for si, raw in enumerate(self.listener_raw):
            if raw is None:
                # plain listen = listenH = listenR with `const $ return True`
                # (:216-219): a name without a typed listener still reaches a
                # handler thread, which only logs "No listener with name"
                # (:240-244) and ends
                missing = [k for k in kinds if k not in self.listener_sets[si]]
                if missing and no_listener is None:
                    no_listener = self.label()
                    self.bind(no_listener)
                    self._emit(isa.OP_END)
                for k in missing:
                    self.listener_sets[si][k] = no_listener
                continue
            typed = self.listener_sets[si]
            entries: Dict[int, Label] = {}
            for k in kinds:
                entry = self.label()
                accept = self.label()
                self.bind(entry)
                c = Code(self)
                raw(c, accept)
                c.end()  # falling off the raw body = return False
                self.bind(accept)
                if k in typed:
                    c.seti(3, k).jmp(typed[k])
                else:
                    c.end()
                entries[k] = entry
            self.listener_sets[si] = entries

    def defer(self, fn: Callable[[], None]) -> None:
        self._deferred.append(fn)

    # -------------------------------------------------------------- finalize
    def finalize(self):
        while self._deferred:
            fns, self._deferred = self._deferred, []
            for fn in fns:
                fn()
        self._expand_raw_listeners()
        insns = np.zeros((len(self._insns), 2), dtype=np.uint32)
        for i, (w0, imm) in enumerate(self._insns):
            if isinstance(imm, Label):
                if imm.pc is None:
                    raise ValueError(f"unbound label {imm.name}")
                imm = imm.pc
            insns[i, 0] = w0
            insns[i, 1] = np.uint32(int(imm) & 0xFFFFFFFF)
        if os.environ.get("TW_FUSE_PAIRS", "1") != "0":
            _fuse_pairs(insns)
        nk = max(1, len(self.msg_kinds))
        ls = np.full((max(1, len(self.listener_sets)), nk), isa.PC_NONE, dtype=np.uint32)
        for si, s in enumerate(self.listener_sets):
            for k, lab in s.items():
                if lab.pc is None:
                    raise ValueError(f"unbound listener {lab.name}")
                ls[si, k] = lab.pc | (isa.LPC_INLINE if k in self.listener_inline[si] else 0)
        consts = np.array(self.consts if self.consts else [0], dtype=np.int64)
        return Image(insns=insns, consts=consts, listener_pc=ls, n_msg_kinds=nk,
                     n_listener_sets=len(self.listener_sets), labels=dict(self._labels))


@dataclass
class Image:
    insns: np.ndarray          # [n, 2] uint32 (w0, imm)
    consts: np.ndarray         # int64
    listener_pc: np.ndarray    # [sets, kinds] uint32
    n_msg_kinds: int
    n_listener_sets: int
    labels: Dict[str, Label] = field(default_factory=dict)

    def pc_of(self, name: str) -> int:
        return self.labels[name].pc


class Code:
    """Emitter for one code block (MonadTimed/MonadDialog vocabulary)."""

    def __init__(self, prog: Program):
        self.p = prog

    def _e(self, op, a=0, b=0, imm: Imm = 0):
        self.p._emit(op, a, b, imm)
        return self

    def _lab(self, x) -> Label:
        return x if isinstance(x, Label) else self.p.label(x)

    # ------------------------------------------------------------ control
    def label(self, name=None) -> Label:
        return self.p.label(name)

    def bind(self, lab) -> Label:
        return self.p.bind(self._lab(lab))

    def here(self, name=None) -> Label:
        return self.p.bind(self.p.label(name))

    def jmp(self, target):
        return self._e(isa.OP_JMP, imm=self._lab(target))

    def end(self):
        return self._e(isa.OP_END)

    # ------------------------------------------------------------- timing
    def wait(self, spec: TimeSpec):
        """``wait`` (TimedT.hs:343-355)."""
        if spec.relative:
            return self._e(isa.OP_WAIT_REL, imm=self.p.const(spec.us))
        return self._e(isa.OP_WAIT_ABS, imm=self.p.const(spec.us))

    def wait_reg(self, r: int):
        return self._e(isa.OP_WAIT_REG, r)

    invoke = wait  # invoke t act = wait t >> act (MonadTimed.hs:182-183)

    def sleep_forever(self):
        """``sleepForever = forever (wait (for 100500 minute))`` (Misc.hs:50-51)."""
        top = self.here()
        self._e(isa.OP_WAIT_REL, imm=self.p.const(100500 * 60_000_000))
        return self.jmp(top)

    def now(self, r: int):
        return self._e(isa.OP_NOW, r)

    # ------------------------------------------------------------ threads
    def fork(self, entry, ref: int = 0, node_reg: Optional[int] = None):
        """``fork`` (TimedT.hs:326-342); child gets a copy of r0..r3."""
        b = 0xFFFF if node_reg is None else node_reg
        return self._e(isa.OP_FORK, ref, b, self._lab(entry))

    def fork_(self, entry, node_reg: Optional[int] = None, scratch: int = 3):
        return self.fork(entry, ref=scratch, node_reg=node_reg)

    def schedule(self, spec: TimeSpec, entry, scratch: int = 3):
        """``schedule t act = fork_ (invoke t act)`` (MonadTimed.hs:162-163)."""
        stub = self.p.label()
        target = self._lab(entry)

        def emit():
            self.p.bind(stub)
            c = Code(self.p)
            c.wait(spec)
            c.jmp(target)

        self.p.defer(emit)
        return self.fork_(stub, scratch=scratch)

    def work(self, spec: TimeSpec, entry, ref: int = 2):
        """``work rel act = fork act >>= schedule rel . killThread`` (MonadTimed.hs:201-202)."""
        self.fork(entry, ref=ref)
        killer = self.p.label()

        def emit():
            self.p.bind(killer)
            c = Code(self.p)
            c.kill_thread(ref)
            c.end()

        self.p.defer(emit)
        return self.schedule(spec, killer, scratch=3 if ref != 3 else 1)

    def my_thread_id(self, r: int):
        return self._e(isa.OP_MYTID, r)

    def throw_to(self, ref: int, exc: int, val_reg: int = 0):
        """``throwTo`` (TimedT.hs:357-368): target woken to now, first exception wins."""
        return self._e(isa.OP_THROW_TO, ref, (exc & 0xFF) | ((val_reg & 3) << 8))

    def kill_thread(self, ref: int):
        """``killThread = flip throwTo ThreadKilled`` (MonadTimed.hs:205-206)."""
        return self.throw_to(ref, isa.EXC_THREAD_KILLED)

    def throw(self, exc: int, val_reg: int = 0):
        """``throwM`` in the current thread."""
        return self._e(isa.OP_THROW, 0, (exc & 0xFF) | ((val_reg & 3) << 8))

    def catch_(self, mask: int, handler):
        """Enter ``act `catch` handler``; handler runs outside the frame with
        r0 = exception value, r3 = exception code (TimedT.hs:183-204)."""
        return self._e(isa.OP_CATCH, 0, mask, self._lab(handler))

    def uncatch(self):
        return self._e(isa.OP_UNCATCH)

    def timeout_begin(self, t_us: int, epoch_reg: int = 3):
        """``timeout t act`` (TimedT.hs:370-376): schedule the watchdog (a fork,
        +1 µs), then enter ``act `finally` done := True``."""
        self._e(isa.OP_TMO_BEGIN, epoch_reg, 0, self.p.const(t_us))
        return self._e(isa.OP_TMO_PUSH, epoch_reg)

    def timeout_end(self):
        return self._e(isa.OP_TMO_END)

    # ----------------------------------------------------------- registers
    def seti(self, r: int, v: int):
        if -(1 << 31) <= v < (1 << 31):
            return self._e(isa.OP_SETI, r, 0, v)
        return self._e(isa.OP_SETK, r, 0, self.p.const(v))

    def addi(self, r: int, v: int):
        return self._e(isa.OP_ADDI, r, 0, v)

    def muli(self, r: int, v: int):
        return self._e(isa.OP_MULI, r, 0, v)

    def modi(self, r: int, v: int):
        return self._e(isa.OP_MODI, r, 0, v)

    def mov(self, r: int, s: int):
        return self._e(isa.OP_MOV, r, s)

    def add(self, r: int, s: int):
        return self._e(isa.OP_ADD, r, s)

    def sub(self, r: int, s: int):
        return self._e(isa.OP_SUB, r, s)

    def jeq(self, r, s, target):
        return self._e(isa.OP_JEQ, r, s, self._lab(target))

    def jne(self, r, s, target):
        return self._e(isa.OP_JNE, r, s, self._lab(target))

    def jlt(self, r, s, target):
        return self._e(isa.OP_JLT, r, s, self._lab(target))

    def jle(self, r, s, target):
        return self._e(isa.OP_JLE, r, s, self._lab(target))

    def jeqi(self, r, v, target):
        return self._e(isa.OP_JEQI, r, v & 0xFFFF, self._lab(target))

    def jnei(self, r, v, target):
        return self._e(isa.OP_JNEI, r, v & 0xFFFF, self._lab(target))

    def node(self, r: int):
        return self._e(isa.OP_NODE, r)

    def nload(self, r: int, var: int):
        return self._e(isa.OP_NLOAD, r, var)

    def nstore(self, r: int, var: int):
        return self._e(isa.OP_NSTORE, r, var)

    def nloadx(self, r: int, var: int, node_reg: int):
        return self._e(isa.OP_NLOADX, r, (var & 0xFF) | ((node_reg & 3) << 8))

    def nstorex(self, r: int, var: int, node_reg: int):
        return self._e(isa.OP_NSTOREX, r, (var & 0xFF) | ((node_reg & 3) << 8))

    def user_state_load(self, r: int, var: int, link_reg: int, state_base: int, scratch: int = 2):
        """``userStateR`` (Transfer.hs; examples/socket-state/Main.hs:91-93):
        the state of the connection the handled message came in on.  A
        connection is an incoming link; its state lives in the node vars of a
        state cell node ``state_base + link`` (4 int64, fresh per replica, like
        `mkState` on each accepted socket).  Handler registers hold the
        incoming link in r1."""
        self.mov(scratch, link_reg).addi(scratch, state_base)
        return self.nloadx(r, var, scratch)

    def user_state_store(self, r: int, var: int, link_reg: int, state_base: int, scratch: int = 2):
        self.mov(scratch, link_reg).addi(scratch, state_base)
        return self.nstorex(r, var, scratch)

    # Connections (MonadTransfer.hs:114-152).  A link carries one connection at
    # a time; the sender numbers them: node var `epoch_var` of the sending node
    # is the current connection's number.  Every message is tagged with it
    # (payload + epoch * CONN_TAG), and the receiving side's state cell for the
    # link remembers which connection its state belongs to (cell var 3): a
    # message of a newer connection finds a fresh ``mkState`` (zeros).  So
    # ``close`` only ends the connection -- data already in flight still
    # arrives on the old one, like bytes written before a FIN.
    CONN_TAG = 1 << 16

    def close_conn(self, epoch_var: int, scratch: int = 3):
        """``close addr`` (MonadTransfer.hs:139-142): the next send opens a new
        connection (clobbers `scratch`)."""
        return self.nload(scratch, epoch_var).addi(scratch, 1).nstore(scratch, epoch_var)

    def conn_tag(self, payload_reg: int, epoch_var: int, scratch: int = 3):
        """Tag a payload (< CONN_TAG) with the sender's current connection number."""
        return self.nload(scratch, epoch_var).muli(scratch, self.CONN_TAG).add(payload_reg, scratch)

    def conn_accept(self, state_base: int):
        """Receiving side of a tagged message in a handler (r0 = tagged payload,
        r1 = incoming link): if it belongs to a newer connection than the link's
        state cell, reset the cell (``mkState`` for the accepted socket) and
        record the connection.  Leaves r0 = r3 = the untagged payload, r1 = the
        link, r2 = the state cell node."""
        T = self.CONN_TAG
        self.mov(2, 1).addi(2, state_base)          # r2 = state cell of the link
        self.mov(3, 0).modi(3, T)                   # r3 = payload
        self.sub(0, 3)                              # r0 = connection tag
        self.nloadx(1, 3, 2)                        # r1 = the cell's connection tag
        same = self.p.label()
        self.jeq(1, 0, same)
        self.nstorex(0, 3, 2)                       # a new connection: record it ...
        self.seti(1, 0)
        for var in range(3):                        # ... with a fresh state
            self.nstorex(1, var, 2)
        self.bind(same)
        self.mov(0, 3)                              # r0 = payload
        self.mov(1, 2).addi(1, -state_base)         # r1 = link
        return self

    def trace(self, tag: int, r: int = 0):
        """Checkpoint / logMeasure-style trace record into the node hash."""
        return self._e(isa.OP_TRACE, r, 0, tag)

    # ------------------------------------------------------------ network
    def link(self, r: int, k: int):
        """r = id of this node's k-th outgoing link (the NetworkAddress)."""
        return self._e(isa.OP_LINK, r, 0, k)

    def reply_link(self, r: int, r_in: int = 1):
        """Link back to the peer of an incoming message (``reply``, MonadDialog.hs:177)."""
        return self._e(isa.OP_RLINK, r, r_in)

    def send(self, link_reg: int, kind: Union[str, int], payload_reg: int = 0):
        """``send`` (MonadDialog.hs:154-156) over the emulated transfer:
        dropped -> nothing; else ``schedule (after d) (deliver ..)``."""
        k = self.p.kind(kind) if isinstance(kind, str) else kind
        return self._e(isa.OP_SEND, link_reg, (k & 0xFF) | ((payload_reg & 3) << 8))

    def listen(self, lset: int, owned: bool = False):
        """``listen (AtPort ..)`` (MonadDialog.hs:204-211): bind this node's port."""
        return self._e(isa.OP_LISTEN, 0, 1 if owned else 0, lset)

    def unlisten(self):
        return self._e(isa.OP_UNLISTEN)
