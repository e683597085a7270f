"""A lowered scenario: program image + topology + per-replica tables.

This is what the reference's (absent) PureRpc runner would have been handed:
the scenario (here: handler tables), the ``Delays`` (here: per-link delay/drop
tables drawn host-side, examples/token-ring/Main.hs:73-77) and the generator
seed.  ``Scenario.desc()`` packs it into the C ABI struct of include/timewarp.h.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import isa
from .abi import TwScenarioDesc
from .program import Image


@dataclass
class Topology:
    """Directed links in CSR over source nodes (a NetworkAddress per link)."""

    n_nodes: int
    out_off: np.ndarray   # uint32 [n_nodes + 1]
    dst: np.ndarray       # uint32 [n_links]
    rev: np.ndarray       # uint32 [n_links]

    @property
    def n_links(self) -> int:
        return int(self.dst.shape[0])

    @staticmethod
    def from_out_lists(n_nodes: int, out: Sequence[Sequence[int]]) -> "Topology":
        off = np.zeros(n_nodes + 1, dtype=np.uint32)
        dst: List[int] = []
        for n in range(n_nodes):
            lst = list(out[n]) if n < len(out) else []
            dst.extend(lst)
            off[n + 1] = len(dst)
        dst_a = np.array(dst, dtype=np.uint32)
        src_a = np.repeat(np.arange(n_nodes, dtype=np.uint32), np.diff(off).astype(np.int64))
        # reverse link: the link dst -> src if it exists (first match)
        index: Dict[Tuple[int, int], int] = {}
        for l, (s, d) in enumerate(zip(src_a.tolist(), dst_a.tolist())):
            index.setdefault((s, d), l)
        rev = np.array([index.get((d, s), isa.PC_NONE) for s, d in zip(src_a.tolist(), dst_a.tolist())],
                       dtype=np.uint32)
        return Topology(n_nodes, off, dst_a, rev)

    def src_of(self) -> np.ndarray:
        return np.repeat(np.arange(self.n_nodes, dtype=np.uint32), np.diff(self.out_off).astype(np.int64))


@dataclass
class Scenario:
    name: str
    image: Image
    topo: Topology
    n_replicas: int
    main_pc: int
    main_node: int
    link_table: Optional[np.ndarray] = None   # uint32 [n_links, depth, n_replicas]
    node_vars: Optional[np.ndarray] = None    # int64 [n_nodes, 4]
    main_regs: Optional[np.ndarray] = None    # int64 [n_replicas, 4]
    node_listen: Optional[np.ndarray] = None  # uint32 [n_nodes]: listener set + 1 bound at t=0
    max_slots: int = 64
    queue_capacity: int = 256
    near_horizon_us: int = 10_000_000
    max_timeouts: int = 0
    run_capacity: int = 0
    max_frames: int = 0                       # catch/finally frames per thread (0 = 2)
    msg_bytes: Optional[np.ndarray] = None    # uint32 [n_msg_kinds]: BinaryP wire size per kind
    link_bw: Optional[np.ndarray] = None      # uint64 [n_links]: bytes/s (0 = no transmission time)
    meta: dict = field(default_factory=dict)
    # oracle-only: the reference's live Delays function (kind/lo/hi per link)
    live_kind: Optional[np.ndarray] = None
    live_lo: Optional[np.ndarray] = None
    live_hi: Optional[np.ndarray] = None

    @property
    def n_nodes(self) -> int:
        return self.topo.n_nodes

    @property
    def link_depth(self) -> int:
        return 1 if self.link_table is None else int(self.link_table.shape[1])

    def with_replicas(self, r0: int, r1: int) -> "Scenario":
        """The replica block [r0, r1) (multi-GPU sharding by contiguous blocks)."""
        lt = None if self.link_table is None else np.ascontiguousarray(self.link_table[:, :, r0:r1])
        mr = None if self.main_regs is None else np.ascontiguousarray(self.main_regs[r0:r1])
        s = Scenario(**{**self.__dict__, "n_replicas": r1 - r0, "link_table": lt, "main_regs": mr})
        s.meta = dict(self.meta, replica_offset=self.meta.get("replica_offset", 0) + r0)
        return s

    def desc(self) -> TwScenarioDesc:
        """Pack into tw_scenario_desc; the returned struct keeps its arrays alive."""
        keep = []

        def ptr(a, dtype):
            if a is None:
                return None
            a = np.ascontiguousarray(a, dtype=dtype)
            keep.append(a)
            return a.ctypes.data

        d = TwScenarioDesc()
        d.abi_version = isa.ABI_VERSION
        d.n_replicas = self.n_replicas
        d.n_nodes = self.n_nodes
        d.n_insns = self.image.insns.shape[0]
        d.insns = ptr(self.image.insns, np.uint32)
        d.n_consts = self.image.consts.shape[0]
        d.consts = ptr(self.image.consts, np.int64)
        d.main_pc = self.main_pc
        d.main_node = self.main_node
        d.n_listener_sets = self.image.n_listener_sets
        d.n_msg_kinds = self.image.n_msg_kinds
        d.listener_pc = ptr(self.image.listener_pc, np.uint32)
        d.n_links = self.topo.n_links
        d.out_off = ptr(self.topo.out_off, np.uint32)
        d.link_dst = ptr(self.topo.dst if self.topo.n_links else np.zeros(1, np.uint32), np.uint32)
        d.link_rev = ptr(self.topo.rev if self.topo.n_links else np.zeros(1, np.uint32), np.uint32)
        d.link_depth = self.link_depth
        if self.link_table is not None:
            assert self.link_table.shape == (self.topo.n_links, self.link_depth, self.n_replicas)
        d.link_table = ptr(self.link_table, np.uint32)
        d.node_vars = ptr(self.node_vars, np.int64)
        d.main_regs = ptr(self.main_regs, np.int64)
        d.node_listen = ptr(self.node_listen, np.uint32)
        d.max_slots = self.max_slots
        d.queue_capacity = self.queue_capacity
        d.near_horizon_us = self.near_horizon_us
        d.max_timeouts = self.max_timeouts
        d.run_capacity = self.run_capacity
        d.max_frames = self.max_frames
        if (self.msg_bytes is None) != (self.link_bw is None):
            raise ValueError("msg_bytes and link_bw go together")
        if self.msg_bytes is not None:
            assert self.msg_bytes.shape == (self.image.n_msg_kinds,)
            assert self.link_bw.shape == (self.topo.n_links,)
        d.msg_bytes = ptr(self.msg_bytes, np.uint32)
        d.link_bw = ptr(self.link_bw, np.uint64)
        d._keep = keep  # type: ignore[attr-defined]
        return d
