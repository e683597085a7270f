"""A CPU stand-in for one rank's LP engine (tests only).

It speaks both window protocols of timewarp.dist -- the host-driven one
(window / take_outbox / inject, dist.lp_loop) and the device-driven one
(exchange_tensors / loop_begin / tick / tick_import / tick_end / progress,
dist.lp_loop_device, with the same send/recv block layout and reduction
words as tw_lp_tick) -- over a toy node-partitioned model, so the loops and
their collectives can be checked at world_size 2 over gloo without a GPU.

The model: node n processing event (t, p) adds mix(n, t, p) to its hash and,
while p > 0, sends (t + L + d(n, p), p - 1) to node (31 n + 7 p) mod N.  Every
send goes through a delivery record (also to a local node), as in LP mode.
A tick processes at most `budget` events per node, so windows can take
several ticks (the rerun path).
"""
import heapq

import numpy as np

from timewarp.engine import LP_RECORD_DTYPE, T_INF

M64 = (1 << 64) - 1


def mix(n, t, p):
    z = (n * 0x9E3779B97F4A7C15 + t * 0xBF58476D1CE4E5B9 + p * 0x94D049BB133111EB) & M64
    z ^= z >> 31
    return (z * 0xD6E8FEB86659FD93) & M64


class StandinLP:
    def __init__(self, n_nodes, lp_begin, lp_count, lookahead, budget=1 << 30, seeds=None, overflow_tick=None):
        self.N, self.b0, self.n, self.L, self.budget = n_nodes, lp_begin, lp_count, lookahead, budget
        # overflow_tick: at that tick this rank reports an inbox overflow (bit 1),
        # as tw_lp_tick does when a node's inbox is full
        self.overflow_tick = overflow_tick
        self.seeds = seeds if seeds is not None else [(i, (i % 7) * 100, 8) for i in range(0, n_nodes, 3)]
        self.reset()

    # ---- shared
    def reset(self):
        self.q = {n: [] for n in range(self.b0, self.b0 + self.n)}
        for node, t, p in self.seeds:
            if self.b0 <= node < self.b0 + self.n:
                heapq.heappush(self.q[node], (t, p))
        self.hash = np.zeros(self.N, np.uint64)
        self.events = 0
        self.out = []      # records produced (not yet routed)
        self.inbox = []    # records waiting for a window's first tick
        return self

    def _local(self, dst):
        return self.b0 <= dst < self.b0 + self.n

    def _run(self, t_end_excl, budget):
        """process events with t < t_end_excl, at most `budget` per node;
        returns whether some node still has such events"""
        active = False
        for node, q in self.q.items():
            k = 0
            while q and q[0][0] < t_end_excl:
                if k == budget:
                    active = True
                    break
                t, p = heapq.heappop(q)
                self.hash[node] = np.uint64((int(self.hash[node]) + mix(node, t, p)) & M64)
                self.events += 1
                k += 1
                if p > 0:
                    dst = (31 * node + 7 * p) % self.N
                    self.out.append((t + self.L + ((13 * node + p) % 5) * 100, p - 1, dst, node))
        return active

    def _next(self):
        return min((q[0][0] for q in self.q.values() if q), default=T_INF)

    def _push(self, rec):
        t, p, dst, _ = rec
        heapq.heappush(self.q[dst], (t, p))

    def results(self):
        return self.events, self.hash

    # ---- host-driven windows (dist.lp_loop)
    def window(self, t_end_excl):
        while self._run(t_end_excl, self.budget):
            pass
        foreign = []
        for r in self.out:
            (self._push(r) if self._local(r[2]) else foreign.append(r))
        self.out = foreign
        return self._next(), len(foreign)

    def launch_ms(self):
        return np.zeros(1)

    def take_outbox(self):
        a = np.zeros(len(self.out), LP_RECORD_DTYPE)
        for i, (t, p, dst, src) in enumerate(self.out):
            a[i] = (t, p, 0, 0, src, dst)
        self.out = []
        return a

    def inject(self, recs):
        for r in recs:
            self._push((int(r["t_arr"]), int(r["payload"]), int(r["dst"]), int(r["src"])))
        return self._next()

    # ---- device-driven windows (dist.lp_loop_device), tw_lp_tick's protocol
    def set_stream(self, s):
        return self

    def exchange_setup(self, world, rank, starts, *ptrs):
        assert world == 1
        self.world, self.rank, self.starts = 1, 0, np.asarray(starts)
        self.bufs = None
        return self

    def exchange_tensors(self, world, rank, starts, send, recv, cap, red):
        self.world, self.rank, self.starts, self.cap = world, rank, np.asarray(starts), cap
        self.bufs = (send.numpy().view(LP_RECORD_DTYPE), recv.numpy().view(LP_RECORD_DTYPE), red.numpy())
        return self

    def loop_begin(self):
        self.T, self.windows, self.ticks, self.fresh, self.done, self.rec_min = 0, 0, 0, True, False, T_INF
        self.active, self.err = False, 0
        return self

    def tick(self):
        if self.done:
            return
        if self.fresh:  # records are drained only at a window's first tick
            for r in self.inbox:
                self._push(r)
            self.inbox = []
        self.active = self._run(self.T + self.L, self.budget)
        if self.overflow_tick is not None and self.ticks == self.overflow_tick:
            self.err |= 1
        for r in self.out:
            if self._local(r[2]):
                self.inbox.append(r)
                self.rec_min = min(self.rec_min, r[0])
            else:
                g = int(np.searchsorted(self.starts, r[2], side="right") - 1)
                send = self.bufs[0]
                base = g * (self.cap + 1)
                k = int(send[base]["t_arr"])  # header: the count in the first word
                assert k < self.cap
                send[base + 1 + k] = (r[0], r[1], 0, 0, r[3], r[2])
                send[base]["t_arr"] = k + 1
        self.out = []

    def tick_import(self):
        if self.bufs is None:
            red = self._red = np.zeros(4, np.int64)
        else:
            red = self.bufs[2]
        red[2] = -self.err  # the overflow bits, reduced with MIN like the other words
        if self.done:
            red[0], red[1] = T_INF, 0
            return
        if self.bufs is not None and self.world > 1:
            recv = self.bufs[1]
            for g in range(self.world):
                base = g * (self.cap + 1)
                for k in range(int(recv[base]["t_arr"])):
                    r = recv[base + 1 + k]
                    self.inbox.append((int(r["t_arr"]), int(r["payload"]), int(r["dst"]), int(r["src"])))
                    self.rec_min = min(self.rec_min, int(r["t_arr"]))
        red[0] = min(self._next(), self.rec_min)
        red[1] = -int(self.active)

    def tick_end(self):
        if self.done:
            return
        red = self._red if self.bufs is None else self.bufs[2]
        self.ticks += 1
        if self.bufs is not None and self.world > 1:
            for g in range(self.world):
                self.bufs[0][g * (self.cap + 1)]["t_arr"] = 0
        if red[2] < 0:  # some rank overflowed: every rank stops at this tick
            self.err |= int(-red[2]) | 16
            self.done = True
            return
        if red[1] < 0:
            self.fresh = False
            return
        self.windows += 1
        if int(red[0]) >= T_INF:
            self.T, self.done = T_INF, True
            return
        self.T, self.fresh, self.rec_min = int(red[0]), True, T_INF

    def progress(self):
        class S:
            pass

        s = S()
        s.windows, s.ticks, s.t, s.done, s.err = self.windows, self.ticks, self.T, int(self.done), self.err
        return s

    def run_windows(self, max_ticks):
        while self.ticks < max_ticks and not self.done:
            self.tick()
            self.tick_import()
            self.tick_end()
        return self.progress()
