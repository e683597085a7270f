// tw_dev.hpp — device-side definitions shared by the HIP kernels of
// libtimewarp.so (engine.hip: lane-per-replica and node-partitioned kernels;
// wave.hip: wave-per-replica kernel): the thread record, the per-replica
// scalar block, the device context and the hash terms.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/timewarp.h"

#ifndef TW_RUNS
#define TW_RUNS 4               // monotone far-queue runs per replica
#endif

// Explicit address spaces: generic (flat) pointers would make every HBM and
// LDS access a flat_* instruction that waits on both memory counters.
#if defined(__HIP_DEVICE_COMPILE__)
#define GAS __attribute__((address_space(1)))
#define LAS __attribute__((address_space(3)))
#else
#define GAS
#define LAS
#endif

namespace tw {

template <class T>
__device__ __forceinline__ T GAS* gp(T* p) {
    return (T GAS*)p;
}

// ------------------------------------------------------------------ layout
// Thread slot record: 64 B, [slot][replica].
//  w0: pc:16 | nfr:4 | flags:6 | exc_code:6
//  w1: node   w2: tid   w3: wake_seq (0 = not queued)
//  f0, f1: the two outermost frames (mask:16 << 16 | pc:16; mask 0 = finally
//          frame of timeout epoch pc); frames 2.. live in the per-slot
//          overflow area fx (TimedT's handler list, TimedT.hs:84,198)
//  xl, xh: pending async exception value (int64, TimedT.hs:113,359)
//  r0..r3: int64 registers
struct Th {
    uint32_t w0, w1, w2, w3;
    uint32_t f0, f1, xl, xh;
    int64_t r0, r1, r2, r3;
};
#define FL_SHIFT 20u   // flags field of w0
#define EXC_SHIFT 26u  // exception-code field of w0

#define F_STARTED 1u
#define F_MAIN 2u
#define F_PHANTOM 4u   // LP mode: a delivery record's stand-in for the deliverer's wake pop
#define F_OWNS 8u      // has bound its node with an owned listener (checked at death)
#define F_NEARQ 16u    // its live queue entry is in the on-chip near heap

__device__ __forceinline__ uint32_t th_pc(const Th& t) { return t.w0 & 0xFFFFu; }
__device__ __forceinline__ void th_set_pc(Th& t, uint32_t pc) { t.w0 = (t.w0 & 0xFFFF0000u) | (pc & 0xFFFFu); }
__device__ __forceinline__ uint32_t th_nfr(const Th& t) { return (t.w0 >> 16) & 15u; }
__device__ __forceinline__ void th_set_nfr(Th& t, uint32_t n) { t.w0 = (t.w0 & ~(15u << 16)) | (n << 16); }
__device__ __forceinline__ uint32_t th_flags(const Th& t) { return (t.w0 >> FL_SHIFT) & 0x3Fu; }
__device__ __forceinline__ void th_or_flags(Th& t, uint32_t f) { t.w0 |= (f & 0x3Fu) << FL_SHIFT; }
__device__ __forceinline__ void th_clr_flags(Th& t, uint32_t f) { t.w0 &= ~((f & 0x3Fu) << FL_SHIFT); }
__device__ __forceinline__ uint32_t th_exc(const Th& t) { return t.w0 >> EXC_SHIFT; }
__device__ __forceinline__ void th_set_exc(Th& t, uint32_t c) {
    t.w0 = (t.w0 & ((1u << EXC_SHIFT) - 1u)) | (c << EXC_SHIFT);
}
__device__ __forceinline__ int64_t th_xval(const Th& t) { return (int64_t)(((uint64_t)t.xh << 32) | t.xl); }
__device__ __forceinline__ void th_set_xval(Th& t, int64_t v) {
    t.xl = (uint32_t)v;
    t.xh = (uint32_t)((uint64_t)v >> 32);
}

enum {
    SC_NOW, SC_FINAL_T, SC_EVENTS, SC_DELIVERED, SC_DROPPED, SC_UNDELIV, SC_THREADS, SC_SEQ, SC_TIDC,
    SC_LIVE, SC_NEAR_N, SC_FAR_N, SC_STATUS, SC_MAIN_EXC, SC_PENDING_MAIN, SC_FREE_N, SC_FTOP, SC_BUMP,
    SC_TMO_CTR, SC_RH0, SC_RC0 = SC_RH0 + TW_RUNS, SC_TRACE_N = SC_RC0 + TW_RUNS,
    // LP: this window's due run of a heavy lane (tw_lp_due): count, head, seq base
    SC_DUE_N, SC_DUE_H, SC_DUE_SEQ, SC_COUNT
};

#define SC_LP_STRIDE 32  // an LP lane's scalar block: 256 B, two 128-B lines
static_assert(SC_COUNT <= SC_LP_STRIDE, "LP scalar block too small");

struct Dev {
    // shape
    uint32_t R, S, Q, N, L, D, T, Cr;
    uint32_t n_insns, n_consts, n_sets, n_kinds;
    int64_t horizon;
    uint64_t RQ;         // quad stride of the thread records: S * R (records are [quad][slot][replica])
    // scenario (shared by all replicas)
    const uint2* insns;
    const int64_t* consts;
    const uint32_t* lpc;
    const uint32_t* out_off;
    const uint32_t* link_dst;
    const uint32_t* link_rev;
    const uint32_t* link_table;   // [L*D][R] or null
    // per-replica scalars: one [field][replica] block of 64-bit words (SC_*)
    uint64_t* scal;
    // per-replica arrays
    uint4* slots;        // [S][R][4]
    uint32_t* free_stk;  // [S][R] (entries below the register-cached top)
    uint4* far;          // [Q][R]  {t_lo, t_hi, slot, seq}
    uint4* runs;         // [TW_RUNS][Cr][R] monotone FIFO runs (ring buffers)
    uint4* near_spill;   // [NEAR_CAP][R]  near heap between launches
    uint4* dummy;        // sinks of the fixed-shape store tail's unused stores (engine.hip TW_DUMMY_*)
    int64_t* nvars;      // [N*4][R]
    uint64_t* hash;      // [N][R]
    uint32_t* bind;      // [N][R] 0 or set+1
    uint32_t* bind_own;  // [N][R] owner tid or 0xFFFFFFFF
    uint32_t* bind_rel;  // [N][R] tid of the last owner that died (0xFFFFFFFE: none); the
                         // binding is live iff bind != 0 && bind_own != bind_rel
    uint32_t* link_ord;  // [L][R]
    uint8_t* tmo_done;   // [T][R]
    uint32_t* n_active;  // [1]
    // node-partitioned (LP) mode: global lane g = lp0 + r runs node g >> rep_lg of
    // replica g & (2^rep_lg - 1) (node-major; rep_lg = 0 for one partitioned
    // scenario, > 0 for the batched mode tw_lpb_load, where cross-node forks
    // travel as spawn records)
    uint32_t lp0, Ntot, IB, out_cap;
    uint32_t rep_lg, lpb;
    uint32_t sc_lp;      // LP context: scal is [lane][SC_LP_STRIDE] (sc_ix), else [SC_COUNT][R]
    int64_t* rw;         // [RW_COUNT][2^rep_lg] per-replica windows (batched LP device loop), else null
    // per-replica windows: the lanes of a replica in chunks of 2^TW_CHUNK_LG
    // nodes, [chunk][replica]: cw_min = a lower bound of the chunk's lanes'
    // next events (exact except after one of them ran: the chunk is then due
    // and rescanned), cw_mark = the window id a lane of the chunk was last marked in
    int64_t* cw_min;
    uint32_t* cw_mark;
    int64_t lookahead;
    uint64_t* hash_g;    // [Ntot << rep_lg] this context's additions to every node's hash
    uint4* inbox;        // delivery records addressed to local lanes: entry k of lane r at
                         // ib_base(r) + k * ib_stride (x2 quads); [IB][R] without ib_off
    uint32_t* inbox_n;   // [2][R]
    // device loop without phases (dpar): a record for a light lane (<= TW_LIGHT
    // pending) is delivered by the sending lane itself, into inbox buffer
    // (wid + 1) & 1, and drained from buffer wid & 1 at the window's first tick
    // (no tw_lp_pack pass for it); heavy lanes and the host loop use buffer 0
    uint32_t dpar;
    size_t ib_total;     // inbox entries per buffer
    const uint4* link_dsth;  // [L] LP: {link_dst | heavy << 31, its inbox offset (ib_off), its inbox
                             // capacity, 0}: a send delivers without looking the node up
    const uint32_t* ib_off;  // batched mode: [Nloc + 1] per-node capacity prefix (records), or null
    uint4* due;          // same layout: a heavy lane's records due in this window, sorted
    uint4* spawn;        // [TW_SPN][R][4] spawn records (batched mode)
    uint32_t* spawn_n;   // [R]
    uint32_t* heavy;     // [2][R] lanes with more than TW_LIGHT pending records
    uint32_t* heavy_n;   // [2]
    uint64_t* pend_min;  // [1] min time of records left pending by tw_lp_due
    // two-phase windows (batched mode): nodes fed by links shorter than the
    // lookahead (a token-ring observer: 0 µs) run in phase 1 of each window,
    // after every phase-0 node has finished the window; null = one phase
    const uint8_t* phase;  // [Ntot]
    uint32_t has_ph1;
    // exchange carry (device loop): foreign records beyond this tick's block
    // size wait here for the next tick (the window reruns until none is left):
    // [2][carry_cap][2], buffer (ticks & 1) written, the other one read
    uint4* carry;
    uint32_t* carry_n;   // [2]
    uint32_t carry_cap;
    uint4* outbox;       // [out_cap][2] records produced this window
    uint32_t* out_n;     // [1]
    uint64_t* next_t;    // [1] min next-event time (atomicMin)
    uint32_t* lp_err;    // [1] inbox/outbox overflow
    // LP work lists: a launch serves only the nodes of list act_cur (those with
    // a live thread or new delivery records); during window wid a node is
    // marked listed[node] = wid, and the next window's list is compacted from
    // the marks (tw_lp_compact)
    uint32_t* act;       // [2][TW_LP_NB][R]
    uint32_t* act_n;     // [2][TW_LP_NB]
    int64_t* wake;       // [R] device loop: the lane's next event time (INT64_MAX: none); a
                         // window lists only lanes due in it, the others' minimum bounds the next
    uint32_t* listed;    // [R]
    // 256-lane blocks of the work-list scan (TW_SUB): a block is rescanned only
    // when one of its lanes was marked (sb_mark), had lanes listed in the last
    // window (sb_scan, both window ids) or holds a wake due in the window
    // (sb_min: the minimum wake of its lanes left unlisted at its last scan)
    uint32_t* sb_mark;   // [R / TW_SUB]
    uint32_t* sb_scan;   // [R / TW_SUB]
    int64_t* sb_min;     // [R / TW_SUB]
    uint32_t* inlist;    // [R] window id whose work list holds the lane (batched mode: a
                         // spawn target is appended to the running window's list once)
    uint32_t act_cur, wid;
    // device-driven windows (tw_lp_tick): the loop state, WN_* words; null
    // for the host-driven loop (tw_lp_window)
    int64_t* win;
    unsigned long long* prof;  // [P_COUNT] diagnostic build only
    uint4* trace;        // [trace_cap][R][2] TRACE records (tw_set_trace), replica mode
    uint32_t trace_cap;
    // handler stack beyond the record's two frames: [S][R][FXQ] quads (frames 2..)
    uint4* fx;
    uint32_t FXQ, max_frames;
    // BinaryP transmission time (tw_scenario_desc.msg_bytes / link_bw)
    const uint32_t* msg_bytes;  // [n_kinds] or null
    const uint64_t* link_bw;    // [L] or null
    uint32_t tie_mode;          // TW_TIE_*: order of equal-timestamp events
    const uint8_t* pc_cls;      // [n_insns + 1] wave kernel: batch class of each resume pc (classify_pcs)
    // batched LP: [n_sets * n_kinds] 1 where the fork_-dispatched handler of a
    // (listener set, kind) may run data-parallel over a heavy lane's due run
    // (classify_batch, tw_lp_due); null: every due record runs on the lane's chain
    const uint8_t* lpc_bat;
    unsigned long long* bat_ctr;  // [2] batched LP since tw_reset: due records run by tw_lp_due, all due records
    // tw_lp_due_batch (round 6): the light lanes its batched replies were
    // delivered to, marked for the next window only after the window's work
    // list is built (tw_lp_dmark): [2][dmk_cap] by window parity, counts [2]
    uint32_t* dmk;
    uint32_t* dmk_n;
    uint32_t dmk_cap;
    uint32_t wave_k;            // wave kernel: near-queue entries per lane (4, 24 or 32), fixed by tw_load
    // wave kernel, tie mode TW_TIE_PQUEUE: each replica's queue is a binomial
    // MinQueue whose nodes are far[r * Q + i] (entries) + pq_link[r * Q + i]
    // {highest-rank child, next lower-rank sibling}; pq_free its free-node
    // stack, pq_scr the toList scratch of a throwTo rebuild, pq_hdr the queue
    // header between launches (PQ_* words)
    uint2* pq_link;
    uint32_t* pq_free;
    uint4* pq_scr;
    uint32_t* pq_hdr;
};
// index of scalar field f of lane / replica r
__host__ __device__ __forceinline__ size_t sc_ix(const Dev& c, uint32_t f, size_t r) {
    return c.sc_lp ? r * SC_LP_STRIDE + f : (size_t)f * c.R + r;
}

// pqueue header words (per replica, [r * PQ_WORDS + w])
enum { PQ_N, PQ_NFREE, PQ_BUMP, PQ_FLEN, PQ_MIN, PQ_FOREST = PQ_MIN + 4, PQ_WORDS = PQ_FOREST + 32 };

// The key an insertion counter value takes in the queues (equal timestamps pop
// in key order): FIFO (canonical), reverse (LIFO) or a scrambled bijection.
// Every mode maps 0 to 0 and nothing else to 0 (wake_seq 0 = not queued).
// TW_TIE_FORKFIRST: bit 31 set on every key but a forked child's (Lane::next_seq),
// so a child sorts before everything queued at the same time.
__device__ __forceinline__ uint32_t seq_key(uint32_t mode, uint32_t s) {
    if (mode == TW_TIE_FIFO || mode == TW_TIE_PQUEUE) return s;  // (pqueue: seq only names the entry)
    if (mode == TW_TIE_FORKFIRST) return s | 0x80000000u;
    if (mode == TW_TIE_LIFO) return 0u - s;
    uint32_t x = s;  // xorshift-multiply: a bijection of u32 with x(0) = 0
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}
// BinaryP transmission time of a message of `kind` over `link` (µs, rounded up)
__device__ __forceinline__ int64_t tx_us(const Dev& c, uint64_t link, uint32_t kind) {
    if (!c.msg_bytes || !c.link_bw || kind >= c.n_kinds) return 0;
    const uint64_t bw = gp(c.link_bw)[link];
    if (!bw) return 0;
    return (int64_t)(((uint64_t)gp(c.msg_bytes)[kind] * 1000000ull + bw - 1) / bw);
}

// LP device-driven window words (Dev::win)
// WN_XMAX: the largest per-rank record demand of one tick since the host last
// cleared it (from the all-reduced words, so identical on every rank: the
// ranks agree on the next exchange block size without talking)
// WN_SPN_HERE, WN_REPS, WN_STEP: per-replica windows (Dev::rw) -- a spawn fell
// inside its replica's window (the window reruns); replicas still running
// after the last advance; what tw_lp_ctl decided this tick (RS_*)
enum { WN_T, WN_L, WN_REC_MIN, WN_WINDOWS, WN_TICKS, WN_FLAGS, WN_ACT, WN_WID, WN_PHASE, WN_NT0, WN_SPN_MIN,
       WN_SLEEP_MIN, WN_XMAX, WN_SPN_HERE, WN_REPS, WN_STEP, WN_COUNT };
// Per-replica windows (batched LP, Dev::rw, [RW_*][2^rep_lg]): the window
// machinery (ticks, reruns, phases, work lists) stays common to the batch,
// but every replica's window is [RW_T, RW_T + L) from its own next event, so a
// window covers what its own replica has due, not the union of all replicas'
// event times.  RW_TICK (u64 min, reset every tick): next events of the lanes
// that ran, spawn times; RW_WIN (u64 min, reset with the window): delivery
// records, records a heavy lane left pending, unlisted lanes' wakes; RW_NT0:
// phase 0's next time while phase 1 runs.
enum { RW_T, RW_TICK, RW_WIN, RW_NT0, RW_COUNT };
enum : int64_t { RS_RERUN = 0, RS_PHASE1 = 1, RS_ADVANCE = 2, RS_STOP = 3 };
// reduction words of the device loop (all-reduced with MIN between ranks)
enum { RD_NEXT, RD_ACTIVE, RD_ERR, RD_DEMAND, RD_COUNT };
// spawn record markers in the kind field of an outbox entry pair (message kinds are < 256)
#define TW_SPAWN_KIND 0xFFFFFFFFu
#define TW_SPAWN_CONT 0xFFFFFFFEu
// WN_FRESH: the window's first tick (phase 0); WN_PH1FRESH: phase 1's first tick
enum : int64_t { WN_FRESH = 1, WN_DONE = 2, WN_PH1FRESH = 4 };

// LP inbox addressing (see Dev::inbox)
#define TW_LIGHT 32u   // a lane with at most this many pending records drains them in the event kernel
#define TW_SPN 4u      // spawn records per lane per tick
#define TW_HEAVY_CAP 2048u  // largest per-node inbox (tw_lp_due stages a lane's records in LDS)
// Batched LP: node n's inbox region holds cap(n) records of each of its 2^rep_lg
// replicas.  A light node's records are replica-interleaved (entry k of every
// replica side by side: the event kernel's waves drain 64 replicas' inboxes
// at once); a heavy node's are one contiguous run per replica (entry k at
// rep * cap + k: tw_lp_due and tw_lp_batch read and write one lane's hundreds
// of records as whole cache lines, instead of one 128-KB-strided record each).
__device__ __forceinline__ size_t ib_heavy_base(const Dev& c, uint32_t off, uint32_t cap, uint32_t g) {
    return ((size_t)off << c.rep_lg) + (size_t)(g & ((1u << c.rep_lg) - 1u)) * cap;
}
__device__ __forceinline__ size_t ib_base(const Dev& c, uint32_t r) {
    if (!c.ib_off) return r;
    const uint32_t g = c.lp0 + r, n = (g >> c.rep_lg) - (c.lp0 >> c.rep_lg);
    const uint32_t o0 = gp(c.ib_off)[n], cap = gp(c.ib_off)[n + 1] - o0;
    if (cap > TW_LIGHT) return ib_heavy_base(c, o0, cap, g);
    return ((size_t)o0 << c.rep_lg) + (g & ((1u << c.rep_lg) - 1u));
}
__device__ __forceinline__ size_t ib_stride(const Dev& c, bool heavy) {
    return c.ib_off ? (heavy ? (size_t)1 : (size_t)1 << c.rep_lg) : (size_t)c.R;
}
// the inbox buffer a delivery to a light lane goes to during window wid
__device__ __forceinline__ uint32_t ib_par_in(const Dev& c, bool light) {
    return (c.dpar && c.win && light) ? ((c.wid + 1u) & 1u) : 0u;
}
__device__ __forceinline__ uint32_t ib_cap(const Dev& c, uint32_t r) {
    if (!c.ib_off) return c.IB;
    const uint32_t n = ((c.lp0 + r) >> c.rep_lg) - (c.lp0 >> c.rep_lg);
    return gp(c.ib_off)[n + 1] - gp(c.ib_off)[n];
}

// mark node r for the next window's work list (tw_lp_compact builds the list
// from the marks, in node order within each wave: coalesced node state)
#define TW_SUB_LG 8  // work-list scan blocks of 256 lanes
#define TW_CHUNK_LG 6  // per-replica windows: 64 nodes per chunk
__device__ __forceinline__ size_t cw_idx(const Dev& c, uint32_t r) {  // [chunk][replica] of lane r
    return ((size_t)((r >> c.rep_lg) >> TW_CHUNK_LG) << c.rep_lg) | (r & ((1u << c.rep_lg) - 1u));
}
__device__ __forceinline__ void lp_mark(const Dev& c, uint32_t r, uint32_t wid) {
    gp(c.listed)[r] = wid;
    if (c.rw) gp(c.cw_mark)[cw_idx(c, r)] = wid;
    else gp(c.sb_mark)[r >> TW_SUB_LG] = wid;  // (lanes of one block store the same value)
}
__device__ __forceinline__ void lp_list_next(const Dev& c, uint32_t r) { lp_mark(c, r, c.wid); }
// per-replica window words of lane r's replica (batched LP, Dev::rw)
__device__ __forceinline__ int64_t GAS* rw_at(const Dev& c, int w, uint32_t r) {
    return gp(c.rw) + ((size_t)w << c.rep_lg) + ((c.lp0 + r) & ((1u << c.rep_lg) - 1u));
}
// the last µs of lane r's replica window (INT64_MIN: the replica is done)
__device__ __forceinline__ int64_t rw_tend(const Dev& c, uint32_t r, int64_t L) {
    const int64_t T = *rw_at(c, RW_T, r);
    return T == INT64_MAX ? INT64_MIN : T + L - 1;
}

// ------------------------------------------------------------------ hashing
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
// == tw_term of include/timewarp.h
__device__ __forceinline__ uint64_t term(int64_t t, uint32_t kind, int64_t val) {
    uint64_t v = val ? mix64((uint64_t)val ^ 0x9e3779b97f4a7c15ull) : 0ull;
    return mix64((((uint64_t)t << 20) | kind) ^ v);
}
__device__ __forceinline__ uint64_t term0(int64_t t, uint32_t kind) { return mix64(((uint64_t)t << 20) | kind); }

__device__ __forceinline__ bool tless(int64_t ta, uint32_t sa, int64_t tb, uint32_t sb) {
    return ta < tb || (ta == tb && sa < sb);
}
__device__ __forceinline__ uint4 ent(int64_t t, uint32_t slot, uint32_t seq) {
    return make_uint4((uint32_t)t, (uint32_t)((uint64_t)t >> 32), slot, seq);
}
__device__ __forceinline__ int64_t ent_t(uint4 e) { return (int64_t)(((uint64_t)e.y << 32) | e.x); }


// Stores by a subset of the lanes WITHOUT a branch: exec is narrowed inside
// one asm block.  A lane-conditional `if` would make the compiler treat every
// value merged after it as divergent, and the whole wave-uniform event loop
// would fall into vector registers under exec masking.  Vector-memory ops
// complete in issue order, so later loads of the same words see these stores.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st32(uint32_t GAS* p, uint32_t v, uint64_t mask = 1) {
    uint64_t sv;
    asm volatile("s_mov_b64 %0, exec\n\ts_and_b64 exec, exec, %3\n\tglobal_store_dword %1, %2, off\n\t"
                 "s_mov_b64 exec, %0" : "=&s"(sv) : "v"(p), "v"(v), "s"(mask) : "memory", "scc");
}
__device__ __forceinline__ void st128(uint4 GAS* p, uint4 v, uint64_t mask = 1) {
    uint64_t sv;
    const u32x4 d = {v.x, v.y, v.z, v.w};
    asm volatile("s_mov_b64 %0, exec\n\ts_and_b64 exec, exec, %3\n\tglobal_store_dwordx4 %1, %2, off\n\t"
                 "s_mov_b64 exec, %0" : "=&s"(sv) : "v"(p), "v"(d), "s"(mask) : "memory", "scc");
}
__device__ __forceinline__ void st8(uint8_t GAS* p, uint32_t v, uint64_t mask = 1) {
    uint64_t sv;
    asm volatile("s_mov_b64 %0, exec\n\ts_and_b64 exec, exec, %3\n\tglobal_store_byte %1, %2, off\n\t"
                 "s_mov_b64 exec, %0" : "=&s"(sv) : "v"(p), "v"(v), "s"(mask) : "memory", "scc");
}
__device__ __forceinline__ void atom_add64(unsigned long long GAS* p, uint64_t v, uint64_t mask = 1) {
    uint64_t sv;
    asm volatile("s_mov_b64 %0, exec\n\ts_and_b64 exec, exec, %3\n\tglobal_atomic_add_x2 %1, %2, off\n\t"
                 "s_mov_b64 exec, %0" : "=&s"(sv) : "v"(p), "v"(v), "s"(mask) : "memory", "scc");
}

// wave.hip: the wave-per-replica kernel (geometry TW_GEO_WAVE)
int wave_near_k(uint32_t R);                // near-queue entries per lane (K) for R replicas (tw_load)
size_t wave_spill_entries(uint32_t K);      // near-queue spill entries per replica
hipError_t wave_launch(const Dev& d, const Dev* d_dev, hipStream_t st, int64_t t_end, uint64_t limit,
                       uint32_t budget);

}  // namespace tw
