// engine.hip — MI355X (gfx950) batched TimedT event engine + the C ABI of
// include/timewarp.h.  Built into time-warp_amd/lib/libtimewarp.so.
//
// Replaces the pure-emulation runner of time-warp:
//   launchTimedT / runTimedT   src/Control/TimeWarp/Timed/TimedT.hs:234-304
//   fork / wait / throwTo / timeout               TimedT.hs:326-376
// for R independent replicas of one lowered scenario.
//
// Mapping to the hardware:
//   * one LANE per replica: a replica's event loop is strictly sequential in
//     TimedT (one pop at a time, TimedT.hs:239-263), replicas are independent,
//     so lanes never synchronise and the whole chip streams replicas;
//   * all per-replica HBM state is replica-minor ([index][replica]): while
//     replicas run in lock-step (scenario start-up, identical programs) a
//     wavefront's 64 accesses to "the same" slot/node/queue index coalesce into
//     contiguous 1-4 KiB transactions; when they diverge each lane touches one
//     64-B line per record;
//   * at one wave per SIMD nothing hides latency, so the event loop keeps its
//     working set on chip: TimedT's event queue (a pqueue MinQueue of
//     continuations) becomes an LDS NEAR heap of 64-bit keys (events due within
//     the scenario's horizon) with its root cached in registers, plus monotone
//     FIFO runs and a 4-ary heap in HBM for far events; thread records of
//     near-queued threads live in a write-back LDS cache (LRU), so the common
//     pop -> run -> re-queue cycle never waits on HBM;
//   * every thread has at most one queued event, so throwTo's queue rebuild
//     (TimedT.hs:361-368) becomes an O(1) re-stamp: a fresh (now, seq) entry is
//     pushed (or the near entry re-keyed in place) and a superseded entry is
//     dropped lazily at pop time (slot.wake_seq no longer matches);
//   * the event order is (t, seq) with seq a per-replica insertion counter —
//     bit-identical to the oracle's canonical mode.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/timewarp.h"

#define TW_NEAR_CAP 16          // on-chip queue entries per replica (LDS)
#define TW_WG 256               // lanes per workgroup (4 waves share one program image)
#define TW_RUNS 4               // monotone far-queue runs per replica
#define TW_RC 6                 // write-back thread-record cache entries per lane (LDS)
#define TW_STEP_CAP (1u << 22)  // instructions per thread step (== oracle kStepCap)

// Explicit address spaces: generic (flat) pointers would make every HBM and
// LDS access a flat_* instruction that waits on both memory counters.
#if defined(__HIP_DEVICE_COMPILE__)
#define GAS __attribute__((address_space(1)))
#define LAS __attribute__((address_space(3)))
#else
#define GAS
#define LAS
#endif

// Diagnostic build (-DTW_PROF_LITE, lib/libtimewarp_lite.so): s_memtime cycle
// splits summed into Dev::prof at kernel end (tools/kernel_probe.py).  The
// product build compiles every LITE_* to nothing.
#ifdef TW_PROF_LITE
#define LITE_T(v) uint64_t v = __builtin_amdgcn_s_memtime()
#define LITE_ACC(i, v) (L.lite[(i)] += (uint32_t)(v))
#define LITE_ACCM(i, v) (lite[(i)] += (uint32_t)(v))
#define LITE_WRAP(i, stmt) do { uint64_t _w0 = __builtin_amdgcn_s_memtime(); stmt; LITE_ACCM(i, __builtin_amdgcn_s_memtime() - _w0); } while (0)
#define KLITE_WRAP(i, stmt) do { uint64_t _w0 = __builtin_amdgcn_s_memtime(); stmt; LITE_ACC(i, __builtin_amdgcn_s_memtime() - _w0); } while (0)
#else
#define LITE_T(v) ((void)0)
#define LITE_ACC(i, v) ((void)0)
#define LITE_ACCM(i, v) ((void)0)
#define LITE_WRAP(i, stmt) do { stmt; } while (0)
#define KLITE_WRAP(i, stmt) do { stmt; } while (0)
#endif
#define P_COUNT 16

namespace {

template <class T>
__device__ __forceinline__ T GAS* gp(T* p) {
    return (T GAS*)p;
}

// ------------------------------------------------------------------ layout
// Thread slot record: 64 B, [slot][replica].
//  w0: pc:16 | nfr:2 | flags:6 | exc_code:8
//  w1: node   w2: tid   w3: wake_seq (0 = not queued)
//  f0..f2: frames (mask:16 << 16 | pc:16; mask 0 = finally frame of epoch pc)
//  w7: pending exception value
//  r0..r3: int64 registers
struct Th {
    uint32_t w0, w1, w2, w3;
    uint32_t f0, f1, f2;
    uint32_t w7;
    int64_t r0, r1, r2, r3;
};

#define F_STARTED 1u
#define F_MAIN 2u
#define F_PHANTOM 4u   // LP mode: a delivery record's stand-in for the deliverer's wake pop
#define F_OWNS 8u      // has bound its node with an owned listener (checked at death)
#define F_NEARQ 16u    // its live queue entry is in the on-chip near heap

__device__ __forceinline__ uint32_t th_pc(const Th& t) { return t.w0 & 0xFFFFu; }
__device__ __forceinline__ void th_set_pc(Th& t, uint32_t pc) { t.w0 = (t.w0 & 0xFFFF0000u) | (pc & 0xFFFFu); }
__device__ __forceinline__ uint32_t th_nfr(const Th& t) { return (t.w0 >> 16) & 3u; }
__device__ __forceinline__ void th_set_nfr(Th& t, uint32_t n) { t.w0 = (t.w0 & ~(3u << 16)) | (n << 16); }
__device__ __forceinline__ uint32_t th_flags(const Th& t) { return (t.w0 >> 18) & 0x3Fu; }
__device__ __forceinline__ void th_or_flags(Th& t, uint32_t f) { t.w0 |= (f & 0x3Fu) << 18; }
__device__ __forceinline__ void th_clr_flags(Th& t, uint32_t f) { t.w0 &= ~((f & 0x3Fu) << 18); }
__device__ __forceinline__ uint32_t th_exc(const Th& t) { return t.w0 >> 24; }
__device__ __forceinline__ void th_set_exc(Th& t, uint32_t c) { t.w0 = (t.w0 & 0x00FFFFFFu) | (c << 24); }

// Registers and frames are selected with mask arithmetic, never indexing: a
// select chain over the fields gets folded into an indexed load, which pins
// the whole record in scratch memory.  Register operands are wave-uniform
// (the dispatch is on the whole instruction word), so the masks are scalar.
__device__ __forceinline__ int64_t getr(const Th& t, uint32_t a) {
    const int64_t m0 = -(int64_t)(a == 0), m1 = -(int64_t)(a == 1), m2 = -(int64_t)(a == 2), m3 = -(int64_t)(a == 3);
    return (t.r0 & m0) | (t.r1 & m1) | (t.r2 & m2) | (t.r3 & m3);
}
__device__ __forceinline__ void setr(Th& t, uint32_t a, int64_t v) {
    const int64_t m0 = -(int64_t)(a == 0), m1 = -(int64_t)(a == 1), m2 = -(int64_t)(a == 2), m3 = -(int64_t)(a == 3);
    t.r0 = (v & m0) | (t.r0 & ~m0);
    t.r1 = (v & m1) | (t.r1 & ~m1);
    t.r2 = (v & m2) | (t.r2 & ~m2);
    t.r3 = (v & m3) | (t.r3 & ~m3);
}
__device__ __forceinline__ uint32_t getf(const Th& t, uint32_t i) {
    const uint32_t m0 = 0u - (i == 0), m1 = 0u - (i == 1), m2 = 0u - (i == 2);
    return (t.f0 & m0) | (t.f1 & m1) | (t.f2 & m2);
}
__device__ __forceinline__ void setf(Th& t, uint32_t i, uint32_t v) {
    const uint32_t m0 = 0u - (i == 0), m1 = 0u - (i == 1), m2 = 0u - (i == 2);
    t.f0 = (v & m0) | (t.f0 & ~m0);
    t.f1 = (v & m1) | (t.f1 & ~m1);
    t.f2 = (v & m2) | (t.f2 & ~m2);
}

enum {
    SC_NOW, SC_FINAL_T, SC_EVENTS, SC_DELIVERED, SC_DROPPED, SC_UNDELIV, SC_THREADS, SC_SEQ, SC_TIDC,
    SC_LIVE, SC_NEAR_N, SC_FAR_N, SC_STATUS, SC_MAIN_EXC, SC_PENDING_MAIN, SC_FREE_N, SC_FTOP, SC_BUMP,
    SC_TMO_CTR, SC_RH0, SC_RC0 = SC_RH0 + TW_RUNS, SC_COUNT = SC_RC0 + TW_RUNS
};

struct Dev {
    // shape
    uint32_t R, S, Q, N, L, D, T, Cr;
    uint32_t n_insns, n_consts, n_sets, n_kinds;
    int64_t horizon;
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
    int64_t* nvars;      // [N*4][R]
    uint64_t* hash;      // [N][R]
    uint32_t* bind;      // [N][R] 0 or set+1
    uint32_t* bind_own;  // [N][R] owner tid or 0xFFFFFFFF
    uint32_t* link_ord;  // [L][R]
    uint8_t* tmo_done;   // [T][R]
    uint32_t* n_active;  // [1]
    // node-partitioned (LP) mode: lane r = global node lp0 + r
    uint32_t lp0, Ntot, IB, out_cap;
    int64_t lookahead;
    uint64_t* hash_g;    // [Ntot] this context's additions to every node's hash
    uint4* inbox;        // [IB][R][2] delivery records addressed to local nodes
    uint32_t* inbox_n;   // [R]
    uint4* outbox;       // [out_cap][2] records produced this window
    uint32_t* out_n;     // [1]
    uint64_t* next_t;    // [1] min next-event time (atomicMin)
    uint32_t* lp_err;    // [1] inbox/outbox overflow
    unsigned long long* prof;  // [P_COUNT] diagnostic build only
};

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

enum { ST_CACHE, ST_THROUGH, ST_DEAD };  // store_rec modes

// Six per-lane words with no array behind them: an array written at a per-lane
// index (the LRU victim) is re-rolled by the compiler into scratch stores.
static_assert(TW_RC == 6, "RegVec6 holds the record-cache metadata");
struct RegVec6 {
    uint32_t v0, v1, v2, v3, v4, v5;
    __device__ __forceinline__ void fill(uint32_t x) { v0 = v1 = v2 = v3 = v4 = v5 = x; }
    // per-lane h: mask arithmetic (a select chain would be folded into an
    // indexed load and pin the whole lane state in scratch)
    __device__ __forceinline__ uint32_t at(int h) const {
        return (v0 & (0u - (h == 0))) | (v1 & (0u - (h == 1))) | (v2 & (0u - (h == 2))) |
               (v3 & (0u - (h == 3))) | (v4 & (0u - (h == 4))) | (v5 & (0u - (h == 5)));
    }
    __device__ __forceinline__ void put(int h, uint32_t x) {
        uint32_t m;
        m = 0u - (h == 0); v0 = (x & m) | (v0 & ~m);
        m = 0u - (h == 1); v1 = (x & m) | (v1 & ~m);
        m = 0u - (h == 2); v2 = (x & m) | (v2 & ~m);
        m = 0u - (h == 3); v3 = (x & m) | (v3 & ~m);
        m = 0u - (h == 4); v4 = (x & m) | (v4 & ~m);
        m = 0u - (h == 5); v5 = (x & m) | (v5 & ~m);
    }
    __device__ __forceinline__ int find(uint32_t x) const {
        int h = -1;
        h = v0 == x ? 0 : h;
        h = v1 == x ? 1 : h;
        h = v2 == x ? 2 : h;
        h = v3 == x ? 3 : h;
        h = v4 == x ? 4 : h;
        h = v5 == x ? 5 : h;
        return h;
    }
    __device__ __forceinline__ int argmin() const {
        int h = 0;
        uint32_t b = v0;
        if (v1 < b) { b = v1; h = 1; }
        if (v2 < b) { b = v2; h = 2; }
        if (v3 < b) { b = v3; h = 3; }
        if (v4 < b) { b = v4; h = 4; }
        if (v5 < b) { b = v5; h = 5; }
        return h;
    }
};

template <bool LP>
struct Lane {
    Dev c;  // by value: kernel arguments stay in SGPRs
    uint32_t r;       // replica
    // LDS (lane-offset pointers; element j at [j * TW_WG])
    uint64_t LAS* nk;     // near heap keys: (t - nbase) << 32 | seq
    uint32_t LAS* ns;     // near heap slots
    uint4 LAS* rcd;       // record cache: entry e quad q at [(e*4+q) * TW_WG]
    const uint2 LAS* P;   // program image
    const int64_t LAS* K; // constant pool
    // near heap
    uint32_t near_n;
    int64_t nbase;
    uint64_t nrk;  // cached root key
    uint32_t nrs;  // cached root slot
    // far runs: head index, count, head (t, seq, slot), tail (t, seq)
    uint32_t rh[TW_RUNS], rn[TW_RUNS];
    int64_t rt[TW_RUNS], ut[TW_RUNS];
    uint32_t rs[TW_RUNS], rsl[TW_RUNS], us[TW_RUNS];
    // far heap top
    uint32_t far_n;
    int64_t ft;
    uint32_t fs, fsl;
    // min over far sources (lazily recomputed: a run head reload overlaps the step)
    bool far_dirty;
    int fsrc;  // -1 none, 0..TW_RUNS-1 run, TW_RUNS heap
    int64_t fmt;
    uint32_t fms, fmsl;
    // write-back record cache: tags, LRU stamps, dirty bits
    RegVec6 ctag, cst;
    uint32_t cdirty, clk;
    // free slots: bump pointer + stack with its top in a register
    uint32_t free_n, ftop, bump;
    // replica scalars
    int64_t now, final_t;
    uint32_t seq, tidc, live, status, main_exc, tmo_ctr;
    uint32_t d_ev, d_dl, d_dr, d_ud, d_th;  // this launch's counter increments
#ifdef TW_PROF_LITE
    uint32_t lite[16];  // sel, pre, step, loop, iters, pops, dispatch, tail, store, spawn, yield-enq, throw, die, selmin, load, pop
#endif

    __device__ __forceinline__ size_t ix(size_t i) const { return i * c.R + r; }
    // per-node arrays: replica mode [node][R]; LP mode a lane owns exactly one node
    __device__ __forceinline__ size_t nix(uint32_t node, uint32_t var) const {
        return LP ? ix(var) : ix((size_t)node * 4 + var);
    }
    __device__ __forceinline__ size_t bix(uint32_t node) const { return LP ? ix(0) : ix(node); }
    __device__ __forceinline__ size_t lix(uint64_t link) const { return LP ? (size_t)link : ix(link); }
    __device__ __forceinline__ size_t tix(uint64_t link, uint32_t ord) const {
        size_t i = (size_t)link * c.D + ord % c.D;
        return LP ? i : ix(i);
    }

    __device__ __forceinline__ void fail(uint32_t st) {
        if (status == TW_REP_RUNNING) status = st;
    }

    // ---------------------------------------------------------- near heap (LDS)
    // 4-ary heap of unique 64-bit keys: 16 entries are two levels, the four
    // children of a node are read together (one LDS round trip per level).
    __device__ __forceinline__ uint64_t nkey(int64_t t, uint32_t s) const {
        return ((uint64_t)(t - nbase) << 32) | s;
    }
    __device__ __forceinline__ bool near_fits(int64_t t) const {
        return near_n < TW_NEAR_CAP && t - now < c.horizon && (uint64_t)(t - nbase) < 0xFFFFFFFFull;
    }
    __device__ __forceinline__ void near_sift_up(uint32_t i, uint64_t k, uint32_t s) {
        while (i > 0) {
            uint32_t p = (i - 1) >> 2;
            uint64_t pk = nk[p * TW_WG];
            uint32_t ps = ns[p * TW_WG];
            if (k > pk) break;
            nk[i * TW_WG] = pk;
            ns[i * TW_WG] = ps;
            i = p;
        }
        nk[i * TW_WG] = k;
        ns[i * TW_WG] = s;
        if (i == 0) { nrk = k; nrs = s; }
    }
    __device__ __forceinline__ void near_sift_down(uint32_t i, uint64_t k, uint32_t s) {
        const uint32_t n = near_n;
        for (;;) {
            uint32_t c0 = 4 * i + 1;
            if (c0 >= n) break;
            uint64_t k0 = nk[c0 * TW_WG], k1 = ~0ull, k2 = ~0ull, k3 = ~0ull;
            uint32_t s0 = ns[c0 * TW_WG], s1 = 0, s2 = 0, s3 = 0;
            if (c0 + 1 < n) { k1 = nk[(c0 + 1) * TW_WG]; s1 = ns[(c0 + 1) * TW_WG]; }
            if (c0 + 2 < n) { k2 = nk[(c0 + 2) * TW_WG]; s2 = ns[(c0 + 2) * TW_WG]; }
            if (c0 + 3 < n) { k3 = nk[(c0 + 3) * TW_WG]; s3 = ns[(c0 + 3) * TW_WG]; }
            uint64_t bk = k0;
            uint32_t bs = s0, bi = c0;
            if (k1 < bk) { bk = k1; bs = s1; bi = c0 + 1; }
            if (k2 < bk) { bk = k2; bs = s2; bi = c0 + 2; }
            if (k3 < bk) { bk = k3; bs = s3; bi = c0 + 3; }
            if (k < bk) break;
            nk[i * TW_WG] = bk;
            ns[i * TW_WG] = bs;
            if (i == 0) { nrk = bk; nrs = bs; }
            i = bi;
        }
        nk[i * TW_WG] = k;
        ns[i * TW_WG] = s;
        if (i == 0) { nrk = k; nrs = s; }
    }
    __device__ __forceinline__ void near_push(int64_t t, uint32_t sq, uint32_t slot) {
        near_sift_up(near_n++, nkey(t, sq), slot);
    }
    __device__ __forceinline__ void near_pop() {
        uint32_t n = --near_n;
        if (n == 0) return;
        near_sift_down(0, nk[n * TW_WG], ns[n * TW_WG]);
    }
    // Re-key the live near entry with seq `old_seq` (seqs are unique) to (t, sq).
    __device__ __forceinline__ bool near_rekey(uint32_t old_seq, int64_t t, uint32_t sq, uint32_t slot) {
        for (uint32_t i = 0; i < near_n; ++i) {
            uint64_t ok = nk[i * TW_WG];
            if ((uint32_t)ok == old_seq) {
                uint64_t k = nkey(t, sq);
                if (k < ok) near_sift_up(i, k, slot);
                else near_sift_down(i, k, slot);
                return true;
            }
        }
        return false;
    }
    // Move the near heap to a new time base (keeps (t - nbase) inside 32 bits).
    __device__ void near_rebase(int64_t nb) {
        uint64_t d = (uint64_t)(nb - nbase) << 32;
        for (uint32_t i = 0; i < near_n; ++i) nk[i * TW_WG] -= d;
        nrk -= d;
        nbase = nb;
    }

    // ------------------------------------------------------ far heap (HBM, 4-ary)
    __device__ __forceinline__ uint4 far_ld(uint32_t i) const { return gp(c.far)[ix(i)]; }
    __device__ __forceinline__ void far_st(uint32_t i, uint4 e) const { gp(c.far)[ix(i)] = e; }
    __device__ __forceinline__ void far_push(int64_t t, uint32_t sq, uint32_t slot) {
        if (far_n >= c.Q) { fail(TW_REP_ERR_QUEUE); return; }
        uint32_t i = far_n++;
        while (i > 0) {
            uint32_t p = (i - 1) >> 2;
            uint4 e = far_ld(p);
            if (!tless(t, sq, ent_t(e), e.w)) break;
            far_st(i, e);
            i = p;
        }
        far_st(i, ent(t, slot, sq));
        if (i == 0) { ft = t; fs = sq; fsl = slot; far_dirty = true; }
    }
    __device__ __forceinline__ void far_pop() {
        uint32_t n = --far_n;
        far_dirty = true;
        if (n == 0) return;
        uint4 le = far_ld(n);
        int64_t t = ent_t(le);
        uint32_t i = 0;
        for (;;) {
            uint32_t c0 = 4 * i + 1;
            if (c0 >= n) break;
            uint32_t cn = n - c0 < 4 ? n - c0 : 4;
            uint4 e0 = far_ld(c0);
            uint4 e1 = cn > 1 ? far_ld(c0 + 1) : e0;
            uint4 e2 = cn > 2 ? far_ld(c0 + 2) : e0;
            uint4 e3 = cn > 3 ? far_ld(c0 + 3) : e0;
            uint4 b = e0;
            uint32_t best = 0;
            if (cn > 1 && tless(ent_t(e1), e1.w, ent_t(b), b.w)) { b = e1; best = 1; }
            if (cn > 2 && tless(ent_t(e2), e2.w, ent_t(b), b.w)) { b = e2; best = 2; }
            if (cn > 3 && tless(ent_t(e3), e3.w, ent_t(b), b.w)) { b = e3; best = 3; }
            if (!tless(ent_t(b), b.w, t, le.w)) break;
            far_st(i, b);
            if (i == 0) { ft = ent_t(b); fs = b.w; fsl = b.z; }
            i = c0 + best;
        }
        far_st(i, le);
        if (i == 0) { ft = t; fs = le.w; fsl = le.z; }
    }

    // ---------------------------------------------------- far runs (HBM FIFOs)
    // Patience-sorting piles: a far event is appended to the run whose tail is
    // the largest key <= it, so runs stay sorted and pops are O(1) with the next
    // head prefetched.  TimedT scenarios park threads in monotone streams
    // (killers at one absolute time, sleepForever timers, re-stamped victims of
    // a killer sweep), so the heap sees only stragglers.
    __device__ __forceinline__ uint4 GAS* run_at(uint32_t j, uint32_t pos) const {
        return gp(c.runs) + ((size_t)j * c.Cr + pos) * c.R + r;
    }
    __device__ __forceinline__ bool run_push(int64_t t, uint32_t sq, uint32_t slot) {
        if (c.Cr == 0) return false;
        int best = -1, empty = -1;
        int64_t bt = 0;
        uint32_t bs = 0;
#pragma unroll
        for (int j = 0; j < TW_RUNS; ++j) {
            if (rn[j] == 0) {
                if (empty < 0) empty = j;
            } else if (rn[j] < c.Cr && !tless(t, sq, ut[j], us[j])) {
                if (best < 0 || tless(bt, bs, ut[j], us[j])) { best = j; bt = ut[j]; bs = us[j]; }
            }
        }
        int sel = best >= 0 ? best : empty;
        if (sel < 0) return false;
#pragma unroll
        for (int j = 0; j < TW_RUNS; ++j) {
            if (j == sel) {
                uint32_t pos = rh[j] + rn[j];
                if (pos >= c.Cr) pos -= c.Cr;
                *run_at(j, pos) = ent(t, slot, sq);
                if (rn[j] == 0) { rt[j] = t; rs[j] = sq; rsl[j] = slot; far_dirty = true; }
                ut[j] = t; us[j] = sq;
                ++rn[j];
            }
        }
        return true;
    }
    __device__ __forceinline__ void run_pop(int sel) {
        far_dirty = true;
#pragma unroll
        for (int j = 0; j < TW_RUNS; ++j) {
            if (j == sel) {
                rh[j] = rh[j] + 1 == c.Cr ? 0 : rh[j] + 1;
                if (--rn[j]) {  // next head: its latency overlaps this event's step
                    uint4 e = *run_at(j, rh[j]);
                    rt[j] = ent_t(e); rs[j] = e.w; rsl[j] = e.z;
                }
            }
        }
    }
    __device__ __forceinline__ void far_min() {
        far_dirty = false;
        fsrc = -1;
        if (far_n) { fsrc = TW_RUNS; fmt = ft; fms = fs; fmsl = fsl; }
#pragma unroll
        for (int j = 0; j < TW_RUNS; ++j)
            if (rn[j] && (fsrc < 0 || tless(rt[j], rs[j], fmt, fms))) { fsrc = j; fmt = rt[j]; fms = rs[j]; fmsl = rsl[j]; }
    }
    __device__ __forceinline__ void push_far(int64_t t, uint32_t sq, uint32_t slot) {
        if (!run_push(t, sq, slot)) far_push(t, sq, slot);
    }

    // ------------------------------------------------------------- queue
    // Queue the thread at t with a fresh seq; returns true if the entry is on chip.
    __device__ __forceinline__ bool enqueue(Th& th, uint32_t slot, int64_t t) {
        uint32_t s = ++seq;
        if (th.w3 == 0) ++live;
        th.w3 = s;
        if (near_fits(t)) {
            near_push(t, s, slot);
            th_or_flags(th, F_NEARQ);
            return true;
        }
        push_far(t, s, slot);
        th_clr_flags(th, F_NEARQ);
        return false;
    }

    // ------------------------------------------------- thread records (cache)
    __device__ __forceinline__ static void unpack(Th& th, uint4 a, uint4 b, uint4 d, uint4 e) {
        th.w0 = a.x; th.w1 = a.y; th.w2 = a.z; th.w3 = a.w;
        th.f0 = b.x; th.f1 = b.y; th.f2 = b.z; th.w7 = b.w;
        th.r0 = (int64_t)(((uint64_t)d.y << 32) | d.x);
        th.r1 = (int64_t)(((uint64_t)d.w << 32) | d.z);
        th.r2 = (int64_t)(((uint64_t)e.y << 32) | e.x);
        th.r3 = (int64_t)(((uint64_t)e.w << 32) | e.z);
    }
    __device__ __forceinline__ static void pack(const Th& th, uint4& a, uint4& b, uint4& d, uint4& e) {
        a = make_uint4(th.w0, th.w1, th.w2, th.w3);
        b = make_uint4(th.f0, th.f1, th.f2, th.w7);
        d = make_uint4((uint32_t)th.r0, (uint32_t)((uint64_t)th.r0 >> 32), (uint32_t)th.r1,
                       (uint32_t)((uint64_t)th.r1 >> 32));
        e = make_uint4((uint32_t)th.r2, (uint32_t)((uint64_t)th.r2 >> 32), (uint32_t)th.r3,
                       (uint32_t)((uint64_t)th.r3 >> 32));
    }
    __device__ __forceinline__ int cfind(uint32_t slot) const { return ctag.find(slot); }
    __device__ __forceinline__ void ctouch(int h) { cst.put(h, ++clk); }
    __device__ __forceinline__ uint4 GAS* hrec(uint32_t slot) const { return gp(c.slots) + ix(slot) * 4; }
    __device__ __forceinline__ uint4 LAS* crec(int e) const { return rcd + (size_t)e * 4 * TW_WG; }
    // HBM holds a record unless the cache has a (newer) copy.
    __device__ __forceinline__ void load_rec(uint32_t slot, Th& th) {
        int h = cfind(slot);
        if (h >= 0) {
            const uint4 LAS* q = crec(h);
            unpack(th, q[0], q[TW_WG], q[2 * TW_WG], q[3 * TW_WG]);
            ctouch(h);
            return;
        }
        const uint4 GAS* p = hrec(slot);
        unpack(th, p[0], p[1], p[2], p[3]);
    }
    __device__ __forceinline__ void writeback(int e) {
        const uint4 LAS* q = crec(e);
        uint4 a = q[0], b = q[TW_WG], d = q[2 * TW_WG], f = q[3 * TW_WG];
        uint4 GAS* p = hrec(ctag.at(e));
        p[0] = a; p[1] = b; p[2] = d; p[3] = f;
    }
    // ST_CACHE: the thread is queued on chip (it runs again soon) -> keep the
    // record in the cache, dirty; ST_THROUGH: queued far -> write it to HBM and
    // drop any cached copy; ST_DEAD: only the header quad (the tid that
    // invalidates stale refs) is written.
    __device__ __forceinline__ void store_rec(uint32_t slot, const Th& th, int mode) {
        uint4 a, b, d, f;
        pack(th, a, b, d, f);
        int h = cfind(slot);
        if (mode == ST_CACHE) {
            if (h < 0) {  // LRU victim (invalid entries carry stamp 0)
                h = cst.argmin();
                if (cdirty & (1u << h)) writeback(h);
                ctag.put(h, slot);
            }
            uint4 LAS* q = crec(h);
            q[0] = a; q[TW_WG] = b; q[2 * TW_WG] = d; q[3 * TW_WG] = f;
            cdirty |= 1u << h;
            ctouch(h);
            return;
        }
        if (h >= 0) {
            ctag.put(h, 0xFFFFFFFFu);
            cst.put(h, 0);
            cdirty &= ~(1u << h);
        }
        uint4 GAS* p = hrec(slot);
        p[0] = a;
        if (mode == ST_THROUGH) { p[1] = b; p[2] = d; p[3] = f; }
    }
    __device__ __forceinline__ void flush_cache() {
#pragma unroll
        for (int e = 0; e < TW_RC; ++e)
            if (cdirty & (1u << e)) writeback(e);
        cdirty = 0;
    }

    // Free slots: never-used slots come from a bump pointer (no memory read);
    // freed slots form a LIFO stack whose top lives in a register.
    __device__ __forceinline__ uint32_t alloc_slot() {
        if (free_n) {
            uint32_t s = ftop;
            if (--free_n) ftop = gp(c.free_stk)[ix(free_n - 1)];
            return s;
        }
        if (bump < c.S) return bump++;
        fail(TW_REP_ERR_SLOTS);
        return 0xFFFFFFFFu;
    }
    __device__ __forceinline__ void free_slot(uint32_t slot) {
        if (free_n) gp(c.free_stk)[ix(free_n - 1)] = ftop;
        ftop = slot;
        ++free_n;
    }

    // Commutative per-node trace hash: a no-return 64-bit atomic add, so the
    // event's critical path never waits on the node's hash line.
    __device__ __forceinline__ void hash_add(uint32_t node, uint64_t v) {
        unsigned long long GAS* h = LP ? (unsigned long long GAS*)(gp(c.hash_g) + node)
                                       : (unsigned long long GAS*)(gp(c.hash) + ix(node));
        __hip_atomic_fetch_add(h, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ __forceinline__ void hash(uint32_t node, uint32_t kind, int64_t val) {
        hash_add(node, term(now, kind, val));
    }
    // LP mode: append a delivery record for another logical process
    __device__ __forceinline__ void emit(int64_t ta, int64_t payload, uint32_t link, uint32_t kind, uint32_t src,
                                         uint32_t dst) {
        uint32_t i = __hip_atomic_fetch_add(gp(c.out_n), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (i >= c.out_cap) {
            __hip_atomic_fetch_or(gp(c.lp_err), 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        uint4 GAS* o = gp(c.outbox) + (size_t)i * 2;
        o[0] = make_uint4((uint32_t)ta, (uint32_t)((uint64_t)ta >> 32), (uint32_t)payload,
                          (uint32_t)((uint64_t)payload >> 32));
        o[1] = make_uint4(link, kind, src, dst);
    }

    // Create a thread queued at now (fork, TimedT.hs:326-339).  Returns its ref.
    __device__ __forceinline__ bool spawn(uint32_t pc, uint32_t node, int64_t q0, int64_t q1, int64_t q2, int64_t q3,
                                          int64_t& ref) {
        uint32_t s = alloc_slot();
        if (s == 0xFFFFFFFFu) return false;
        Th ch;
        uint32_t tid = tidc++;
        ++d_th;
        ch.w0 = pc & 0xFFFFu;
        ch.w1 = node;
        ch.w2 = tid;
        ch.w3 = 0;
        ch.f0 = ch.f1 = ch.f2 = ch.w7 = 0;
        ch.r0 = q0; ch.r1 = q1; ch.r2 = q2; ch.r3 = q3;
        bool on_chip = enqueue(ch, s, now);
        store_rec(s, ch, on_chip ? ST_CACHE : ST_THROUGH);
        ref = (int64_t)(((uint64_t)tid << 32) | s);
        return true;
    }

    // throwTo (TimedT.hs:357-368): re-stamp target's event to now, first exception wins.
    __device__ __forceinline__ void throw_to(Th& self, uint32_t self_slot, int64_t ref, uint32_t code, int64_t val) {
        uint32_t ts = (uint32_t)ref;
        uint32_t tid = (uint32_t)((uint64_t)ref >> 32);
        if (ts >= c.S) return;
        if (ts == self_slot) {  // the running thread: its record lives in registers
            if (self.w2 != tid) return;
            if (th_exc(self) == 0) { th_set_exc(self, code); self.w7 = (uint32_t)val; }
            return;
        }
        Th t;
        load_rec(ts, t);
        if (t.w2 != tid) return;  // dead (slot free or reused): the map entry is unobservable
        bool on_chip = (th_flags(t) & F_NEARQ) != 0;
        if (t.w3 != 0) {          // queued: wake to now with a fresh seq
            uint32_t s = ++seq;
            if (!(on_chip && near_rekey(t.w3, now, s, ts))) {
                on_chip = near_fits(now);
                if (on_chip) near_push(now, s, ts);
                else push_far(now, s, ts);
            }
            if (on_chip) th_or_flags(t, F_NEARQ);
            else th_clr_flags(t, F_NEARQ);
            t.w3 = s;
        }
        if (th_exc(t) == 0) {
            th_set_exc(t, code);
            t.w7 = (uint32_t)val;
        }
        store_rec(ts, t, on_chip ? ST_CACHE : ST_THROUGH);
    }

    // Thread ends (END or uncaught exception).
    __device__ __forceinline__ void die(Th& th, uint32_t slot) {
        if (th_flags(th) & F_OWNS) {
            uint32_t node = th.w1;
            if (gp(c.bind_own)[bix(node)] == th.w2) {
                gp(c.bind)[bix(node)] = 0;
                gp(c.bind_own)[bix(node)] = 0xFFFFFFFFu;
            }
        }
        th.w2 = 0xFFFFFFFFu;  // invalidate refs to this slot
        th.w3 = 0;
        store_rec(slot, th, ST_DEAD);
        free_slot(slot);
    }

    // Raise `code` in th; true if a catch frame took it (pc set to handler).
    __device__ __forceinline__ bool unwind(Th& th, uint32_t slot, uint32_t code, int64_t val) {
        const uint32_t n = th_nfr(th);
#pragma unroll
        for (int i = TW_MAX_FRAMES - 1; i >= 0; --i) {
            if ((uint32_t)i < n) {
                uint32_t f = i == 0 ? th.f0 : i == 1 ? th.f1 : th.f2;
                uint32_t mask = f >> 16;
                if (mask == 0) {
                    uint32_t e = f & 0xFFFFu;
                    if (e < c.T) gp(c.tmo_done)[ix(e)] = 1;
                } else if (mask & (1u << code)) {
                    th_set_nfr(th, (uint32_t)i);
                    th_set_pc(th, f & 0xFFFFu);
                    th.r0 = val;
                    th.r3 = code;
                    return true;
                }
            }
        }
        th_set_nfr(th, 0);
        if (th_flags(th) & F_MAIN) main_exc = code;
        die(th, slot);
        return false;
    }

    // Run the thread's continuation until it yields or ends (the ContT
    // continuation of TimedT.hs:343-355).  Dispatch is a waterfall over the
    // instruction words present in the wave: readfirstlane picks one, the lanes
    // holding it execute it with op and register operands wave-uniform (scalar
    // branches), the others wait for their turn — lanes in lock-step take one
    // pass per instruction.  Every yielding op funnels into one shared
    // spawn + enqueue tail.
    __device__ __forceinline__ void step(Th& th, uint32_t slot) {
        enum { GO, YIELD, SPAWN, THROWTO, EXIT, STOP };
        th_or_flags(th, F_STARTED);
        uint32_t n = 0;
        uint32_t pc = th_pc(th);
        if (pc >= c.n_insns) { fail(TW_REP_ERR_INSN); store_rec(slot, th, ST_THROUGH); return; }
        uint2 in = P[pc];
        int mode = ST_THROUGH;
        LITE_T(q0t);
#ifdef TW_PROF_LITE
        uint64_t q1t = q0t;
#endif
        for (;;) {
            const uint32_t w = in.x;
            if (w != __builtin_amdgcn_readfirstlane(w)) continue;
            uint32_t uw;  // opaque scalar copy: keeps every decode below on the SALU
            asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(uw) : "v"(w));
            if (++n > TW_STEP_CAP) { fail(TW_REP_ERR_INSN); break; }
            uint2 nx = P[pc + 1];  // prefetch the fall-through instruction (image padded by one)
            const uint32_t op = uw & 0xFFu, a = (uw >> 8) & 3u, b = uw >> 16;
            const int32_t imm = (int32_t)in.y;
            uint32_t npc = pc + 1;
            int act = GO;
            int64_t yt = 0;                               // YIELD: wake time
            uint32_t cpc = 0, cnode = 0;                  // SPAWN: child entry + node
            int64_t q0 = 0, q1 = 0, q2 = 0, q3 = 0;       //        child registers
            int64_t tref = 0, tval = 0;                   // THROWTO target + payload
            uint32_t tcode = 0;
            switch (op) {
            case TW_OP_NOP: break;
            case TW_OP_END: act = EXIT; break;
            case TW_OP_WAIT_REL: yt = now + K[imm]; act = YIELD; break;
            case TW_OP_WAIT_ABS: {
                int64_t t = K[imm];
                yt = t > now ? t : now;
                act = YIELD;
                break;
            }
            case TW_OP_WAIT_REG: {
                int64_t d = getr(th, a);
                yt = now + (d > 0 ? d : 0);
                act = YIELD;
                break;
            }
            case TW_OP_FORK: {
                uint32_t node = b == 0xFFFFu ? th.w1 : (uint32_t)getr(th, b & 3);
                if (LP ? node != th.w1 : node >= c.N) { fail(TW_REP_ERR_INSN); act = STOP; break; }
                cpc = (uint32_t)imm; cnode = node;
                q0 = th.r0; q1 = th.r1; q2 = th.r2; q3 = th.r3;
                act = SPAWN;
                break;
            }
            case TW_OP_MYTID: setr(th, a, (int64_t)(((uint64_t)th.w2 << 32) | slot)); break;
            case TW_OP_THROW_TO:
                tref = getr(th, a); tcode = b & 0xFFu; tval = getr(th, (b >> 8) & 3);
                act = THROWTO;
                break;
            case TW_OP_THROW:
                th_set_pc(th, npc);
                if (!unwind(th, slot, b & 0xFFu, getr(th, (b >> 8) & 3))) return;  // died (record stored)
                npc = th_pc(th);
                break;
            case TW_OP_CATCH: {
                uint32_t nf = th_nfr(th);
                if (nf >= TW_MAX_FRAMES) { fail(TW_REP_ERR_FRAMES); act = STOP; break; }
                setf(th, nf, (b << 16) | ((uint32_t)imm & 0xFFFFu));
                th_set_nfr(th, nf + 1);
                break;
            }
            case TW_OP_UNCATCH: {
                uint32_t nf = th_nfr(th);
                if (nf == 0 || (getf(th, nf - 1) >> 16) == 0) { fail(TW_REP_ERR_INSN); act = STOP; break; }
                th_set_nfr(th, nf - 1);
                break;
            }
            case TW_OP_SETI: setr(th, a, imm); break;
            case TW_OP_SETK: setr(th, a, K[imm]); break;
            case TW_OP_ADDI: setr(th, a, getr(th, a) + imm); break;
            case TW_OP_MULI: setr(th, a, getr(th, a) * imm); break;
            case TW_OP_MOV: setr(th, a, getr(th, b & 3)); break;
            case TW_OP_ADD: setr(th, a, getr(th, a) + getr(th, b & 3)); break;
            case TW_OP_SUB: setr(th, a, getr(th, a) - getr(th, b & 3)); break;
            case TW_OP_MODI: {
                int64_t m = getr(th, a) % imm;
                setr(th, a, m < 0 ? m + imm : m);
                break;
            }
            case TW_OP_JMP: npc = (uint32_t)imm; break;
            case TW_OP_JEQ: if (getr(th, a) == getr(th, b & 3)) npc = (uint32_t)imm; break;
            case TW_OP_JNE: if (getr(th, a) != getr(th, b & 3)) npc = (uint32_t)imm; break;
            case TW_OP_JLT: if (getr(th, a) < getr(th, b & 3)) npc = (uint32_t)imm; break;
            case TW_OP_JLE: if (getr(th, a) <= getr(th, b & 3)) npc = (uint32_t)imm; break;
            case TW_OP_JEQI: if (getr(th, a) == (int64_t)(int16_t)b) npc = (uint32_t)imm; break;
            case TW_OP_JNEI: if (getr(th, a) != (int64_t)(int16_t)b) npc = (uint32_t)imm; break;
            case TW_OP_NOW: setr(th, a, now); break;
            case TW_OP_NODE: setr(th, a, th.w1); break;
            case TW_OP_NLOAD: setr(th, a, gp(c.nvars)[nix(th.w1, b & 3)]); break;
            case TW_OP_NSTORE: gp(c.nvars)[nix(th.w1, b & 3)] = getr(th, a); break;
            case TW_OP_NLOADX:
            case TW_OP_NSTOREX: {
                uint64_t node = (uint64_t)getr(th, (b >> 8) & 3);
                if (LP ? node != th.w1 : node >= c.N) { fail(TW_REP_ERR_INSN); act = STOP; break; }
                int64_t GAS* v = &gp(c.nvars)[nix((uint32_t)node, b & 3)];
                if (op == TW_OP_NLOADX) setr(th, a, *v);
                else *v = getr(th, a);
                break;
            }
            case TW_OP_LINK: setr(th, a, (int64_t)gp(c.out_off)[th.w1] + imm); break;
            case TW_OP_RLINK: {
                uint64_t l = (uint64_t)getr(th, b & 3);
                if (l >= c.L) { fail(TW_REP_ERR_INSN); act = STOP; break; }
                setr(th, a, (int64_t)gp(c.link_rev)[l]);
                break;
            }
            case TW_OP_SEND: {  // schedule (after d) (deliver ..) unless the link drops it
                uint64_t link = (uint64_t)getr(th, a);
                if (link >= c.L) { fail(TW_REP_ERR_INSN); act = STOP; break; }
                uint32_t kind = b & 0xFFu;
                int64_t payload = getr(th, (b >> 8) & 3);
                uint32_t ord = gp(c.link_ord)[lix(link)];
                gp(c.link_ord)[lix(link)] = ord + 1;
                uint32_t e = c.link_table ? gp(c.link_table)[tix(link, ord)] : 0u;
                if (e & TW_LINK_DROP) {
                    ++d_dr;
                    hash(th.w1, TW_KIND_DROP | kind, payload);
                    break;
                }
                if (LP) {
                    // the deliverer `schedule (after d) deliver` is accounted here (start pop
                    // at now, wake pop at now+d, both at this node) and its delivery travels
                    // as a record: the receiver checks its binding at now+d
                    int64_t dly = (int64_t)(e & 0x7FFFFFFFu);
                    if (dly < c.lookahead) { fail(TW_REP_ERR_INSN); act = STOP; break; }
                    int64_t ta = now + dly;
                    hash_add(th.w1, term0(now, TW_KIND_RESUME | TW_PC_DELIVER_STUB) +
                                        term0(ta, TW_KIND_RESUME | (TW_PC_DELIVER_STUB + 1)));
                    d_ev += 2;
                    ++d_th;
                    final_t = ta > final_t ? ta : final_t;
                    emit(ta, payload, (uint32_t)link, kind, th.w1, gp(c.link_dst)[link]);
                    yt = now + 1;
                    act = YIELD;
                    break;
                }
                cpc = TW_PC_DELIVER_STUB; cnode = th.w1;
                q0 = payload; q1 = (int64_t)link; q2 = (int64_t)(e & 0x7FFFFFFFu); q3 = (int64_t)kind;
                act = SPAWN;
                break;
            }
            case TW_OP_DELIVER: {  // listener dispatch, ForkStrategy fork_ (MonadDialog.hs:232-256,317)
                uint64_t link = (uint64_t)th.r1;
                uint32_t kind = (uint32_t)th.r3;
                uint32_t dst = gp(c.link_dst)[link];
                uint32_t set = gp(c.bind)[bix(dst)];
                uint32_t lpc = TW_PC_NONE;
                if (set && kind < c.n_kinds) lpc = gp(c.lpc)[(size_t)(set - 1) * c.n_kinds + kind];
                if (lpc == TW_PC_NONE) {
                    ++d_ud;
                    hash(dst, TW_KIND_UNDELIV | kind, th.r0);
                    if (LP) act = EXIT;  // the phantom deliverer ends here
                    break;
                }
                ++d_dl;
                hash(dst, TW_KIND_RECV | kind, th.r0);
                cpc = lpc; cnode = dst;
                q0 = th.r0; q1 = (int64_t)link; q2 = LP ? th.r2 : (int64_t)th.w1; q3 = (int64_t)kind;
                act = SPAWN;
                break;
            }
            case TW_OP_LISTEN:
                if ((uint32_t)imm >= c.n_sets) { fail(TW_REP_ERR_INSN); act = STOP; break; }
                gp(c.bind)[bix(th.w1)] = (uint32_t)imm + 1;
                gp(c.bind_own)[bix(th.w1)] = b ? th.w2 : 0xFFFFFFFFu;
                if (b) th_or_flags(th, F_OWNS);
                break;
            case TW_OP_UNLISTEN:
                gp(c.bind)[bix(th.w1)] = 0;
                gp(c.bind_own)[bix(th.w1)] = 0xFFFFFFFFu;
                break;
            case TW_OP_TRACE: hash(th.w1, TW_KIND_TRACE | ((uint32_t)imm & 0xFFFFu), getr(th, a)); break;
            case TW_OP_TMO_BEGIN: {  // schedule (after t) watchdog (TimedT.hs:373-375)
                if (tmo_ctr >= c.T) { fail(TW_REP_ERR_INSN); act = STOP; break; }
                uint32_t e = tmo_ctr++;
                gp(c.tmo_done)[ix(e)] = 0;
                setr(th, a, e);
                cpc = TW_PC_WATCHDOG_STUB; cnode = th.w1;
                q0 = (int64_t)(((uint64_t)th.w2 << 32) | slot); q1 = (int64_t)e; q2 = K[imm]; q3 = 0;
                act = SPAWN;
                break;
            }
            case TW_OP_TMO_PUSH: {
                uint32_t nf = th_nfr(th);
                if (nf >= TW_MAX_FRAMES) { fail(TW_REP_ERR_FRAMES); act = STOP; break; }
                setf(th, nf, (uint32_t)getr(th, a) & 0xFFFFu);
                th_set_nfr(th, nf + 1);
                break;
            }
            case TW_OP_TMO_END: {
                uint32_t nf = th_nfr(th);
                if (nf == 0 || (getf(th, nf - 1) >> 16) != 0) { fail(TW_REP_ERR_INSN); act = STOP; break; }
                uint32_t ep = getf(th, nf - 1) & 0xFFFFu;
                th_set_nfr(th, nf - 1);
                if (ep < c.T) gp(c.tmo_done)[ix(ep)] = 1;
                break;
            }
            case TW_OP_TMO_FIRE: {
                uint64_t e = (uint64_t)th.r1;
                if (e < c.T && !gp(c.tmo_done)[ix(e)]) {
                    tref = th.r0; tcode = TW_EXC_TIMEOUT; tval = 0;
                    act = THROWTO;
                }
                break;
            }
            default:
                fail(TW_REP_ERR_INSN);
                act = STOP;
                break;
            }
            th_set_pc(th, npc);
#ifdef TW_PROF_LITE
            q1t = __builtin_amdgcn_s_memtime();
            LITE_ACCM(6, q1t - q0t);
            q0t = q1t;
#endif
            if (act == EXIT) {
                LITE_WRAP(12, die(th, slot));
                return;
            }
            if (act == THROWTO) {
                LITE_WRAP(11, throw_to(th, slot, tref, tcode, tval));
                act = GO;
            }
            if (act == SPAWN) {  // fork (TimedT.hs:326-342): child at now, parent waits 1 µs
                int64_t ref;
                bool ok;
                LITE_WRAP(9, ok = spawn(cpc, cnode, q0, q1, q2, q3, ref));
                if (!ok) break;
                if (op == TW_OP_FORK) setr(th, a, ref);
                if (LP && op == TW_OP_DELIVER) {
                    // the deliverer's resume pop (at now+1, on the sending node), then it ends
                    hash_add((uint32_t)th.r2, term0(now + 1, TW_KIND_RESUME | (TW_PC_DELIVER_STUB + 2)));
                    ++d_ev;
                    final_t = now + 1 > final_t ? now + 1 : final_t;
                    die(th, slot);
                    return;
                }
                yt = now + 1;
                act = YIELD;
            }
            if (act == YIELD) {
                LITE_WRAP(10, mode = enqueue(th, slot, yt) ? ST_CACHE : ST_THROUGH);
                break;
            }
#ifdef TW_PROF_LITE
            q1t = __builtin_amdgcn_s_memtime();
            LITE_ACCM(7, q1t - q0t);
            q0t = q1t;
#endif
            if (act == STOP || status != TW_REP_RUNNING) break;
            if (npc >= c.n_insns) { fail(TW_REP_ERR_INSN); break; }
            if (npc == pc + 1) in = nx;
            else in = P[npc];
            pc = npc;
        }
#ifdef TW_PROF_LITE
        q1t = __builtin_amdgcn_s_memtime();
        LITE_ACCM(7, q1t - q0t);
#endif
        store_rec(slot, th, mode);
        LITE_ACCM(8, __builtin_amdgcn_s_memtime() - q1t);
    }
};

// ------------------------------------------------------------------ kernels
__global__ void __launch_bounds__(TW_WG) tw_init_kernel(Dev c, uint32_t main_pc, uint32_t main_node,
                                                       const int64_t* main_regs, const int64_t* nv_init,
                                                       const uint32_t* listen_init, int lp_mode) {
    uint32_t r = blockIdx.x * TW_WG + threadIdx.x;
    if (r >= c.R) return;
    // LP mode: lane r is global node g; only the main node's lane holds the main thread
    const uint32_t g = lp_mode ? c.lp0 + r : 0u;
    const bool has_main = !lp_mode || g == main_node;
    for (uint32_t f = 0; f < SC_COUNT; ++f) gp(c.scal)[(size_t)f * c.R + r] = 0;
    gp(c.scal)[(size_t)SC_THREADS * c.R + r] = has_main ? 1 : 0;
    gp(c.scal)[(size_t)SC_TIDC * c.R + r] = 1;
    gp(c.scal)[(size_t)SC_STATUS * c.R + r] = TW_REP_RUNNING;
    gp(c.scal)[(size_t)SC_PENDING_MAIN * c.R + r] = has_main ? 1 : 0;
    gp(c.scal)[(size_t)SC_BUMP * c.R + r] = has_main ? 1 : 0;  // slot 0 = main
    uint4 GAS* p = gp(c.slots) + (size_t)r * 4;  // slot 0
    uint32_t w0 = (main_pc & 0xFFFFu) | (F_MAIN << 18);
    p[0] = make_uint4(w0, main_node, has_main ? 0u : 0xFFFFFFFFu, 0u);
    p[1] = make_uint4(0u, 0u, 0u, 0u);
    int64_t m[4] = {0, 0, 0, 0};
    if (main_regs && !lp_mode)
        for (int i = 0; i < 4; ++i) m[i] = main_regs[(size_t)r * 4 + i];
    p[2] = make_uint4((uint32_t)m[0], (uint32_t)((uint64_t)m[0] >> 32), (uint32_t)m[1], (uint32_t)((uint64_t)m[1] >> 32));
    p[3] = make_uint4((uint32_t)m[2], (uint32_t)((uint64_t)m[2] >> 32), (uint32_t)m[3], (uint32_t)((uint64_t)m[3] >> 32));
    if (lp_mode) {
        if (nv_init)
            for (uint32_t i = 0; i < 4; ++i) gp(c.nvars)[(size_t)i * c.R + r] = nv_init[(size_t)g * 4 + i];
        gp(c.bind_own)[r] = 0xFFFFFFFFu;
        if (listen_init) gp(c.bind)[r] = listen_init[g];
        gp(c.inbox_n)[r] = 0;
        return;
    }
    if (nv_init)
        for (uint32_t i = 0; i < c.N * 4; ++i) gp(c.nvars)[(size_t)i * c.R + r] = nv_init[i];
    for (uint32_t n = 0; n < c.N; ++n) gp(c.bind_own)[(size_t)n * c.R + r] = 0xFFFFFFFFu;
    if (listen_init)
        for (uint32_t n = 0; n < c.N; ++n) gp(c.bind)[(size_t)n * c.R + r] = listen_init[n];
}

// LDS per workgroup: near heap keys + slots, the record cache, then the program
// image and constant pool, so instruction fetch and time constants never
// leave the CU.
__host__ __device__ constexpr size_t fixed_lds_bytes() {
    return (size_t)TW_NEAR_CAP * TW_WG * 12 + (size_t)TW_RC * 4 * TW_WG * 16;
}

template <bool LP>
__global__ void __launch_bounds__(TW_WG) __attribute__((amdgpu_waves_per_eu(1, 2)))
tw_run_kernel(Dev c, int64_t t_end, uint64_t max_events, uint32_t budget) {
    extern __shared__ __attribute__((aligned(16))) uint64_t lds_raw[];
    uint4 LAS* s_rc = (uint4 LAS*)lds_raw;
    uint64_t LAS* s_k = (uint64_t LAS*)(s_rc + TW_RC * 4 * TW_WG);
    uint32_t LAS* s_s = (uint32_t LAS*)(s_k + TW_NEAR_CAP * TW_WG);
    uint2 LAS* s_p = (uint2 LAS*)(s_s + TW_NEAR_CAP * TW_WG);
    int64_t LAS* s_c = (int64_t LAS*)(s_p + c.n_insns + 1);
    {
        for (uint32_t i = threadIdx.x; i <= c.n_insns; i += TW_WG) s_p[i] = gp(c.insns)[i];
        for (uint32_t i = threadIdx.x; i < c.n_consts; i += TW_WG) s_c[i] = gp(c.consts)[i];
        __syncthreads();
    }
    uint32_t r = blockIdx.x * TW_WG + threadIdx.x;
    if (r >= c.R) return;
    uint64_t* sc = gp(c.scal) + r;
    const size_t R = c.R;
    if (sc[SC_STATUS * R] != TW_REP_RUNNING) return;

    Lane<LP> L;
    L.c = c;
    L.r = r;
    L.nk = s_k + threadIdx.x;
    L.ns = s_s + threadIdx.x;
    L.rcd = s_rc + threadIdx.x;
    L.P = s_p;
    L.K = s_c;
    L.ctag.fill(0xFFFFFFFFu);
    L.cst.fill(0);
    L.cdirty = 0;
    L.clk = 0;
    L.now = (int64_t)sc[SC_NOW * R]; L.final_t = (int64_t)sc[SC_FINAL_T * R];
    L.seq = (uint32_t)sc[SC_SEQ * R]; L.tidc = (uint32_t)sc[SC_TIDC * R]; L.live = (uint32_t)sc[SC_LIVE * R];
    const uint32_t near_n0 = (uint32_t)sc[SC_NEAR_N * R];
    L.far_n = (uint32_t)sc[SC_FAR_N * R];
    L.status = (uint32_t)sc[SC_STATUS * R]; L.main_exc = (uint32_t)sc[SC_MAIN_EXC * R];
    L.free_n = (uint32_t)sc[SC_FREE_N * R]; L.ftop = (uint32_t)sc[SC_FTOP * R]; L.bump = (uint32_t)sc[SC_BUMP * R];
    L.tmo_ctr = (uint32_t)sc[SC_TMO_CTR * R];
    const uint64_t events0 = sc[SC_EVENTS * R];
    const uint64_t ev_room64 = max_events > events0 ? max_events - events0 : 0;
    const uint32_t ev_room = ev_room64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)ev_room64;
    L.d_ev = L.d_dl = L.d_dr = L.d_ud = L.d_th = 0;
    L.ft = 0; L.fs = 0; L.fsl = 0;
    if (L.far_n) {
        uint4 e = L.far_ld(0);
        L.ft = ent_t(e); L.fs = e.w; L.fsl = e.z;
    }
#pragma unroll
    for (int j = 0; j < TW_RUNS; ++j) {
        L.rh[j] = (uint32_t)sc[(SC_RH0 + j) * R];
        L.rn[j] = (uint32_t)sc[(SC_RC0 + j) * R];
        L.rt[j] = L.ut[j] = 0;
        L.rs[j] = L.us[j] = L.rsl[j] = 0;
        if (L.rn[j]) {
            uint4 h = *L.run_at(j, L.rh[j]);
            uint32_t tp = L.rh[j] + L.rn[j] - 1;
            if (tp >= c.Cr) tp -= c.Cr;
            uint4 u = *L.run_at(j, tp);
            L.rt[j] = ent_t(h); L.rs[j] = h.w; L.rsl[j] = h.z;
            L.ut[j] = ent_t(u); L.us[j] = u.w;
        }
    }
    L.far_min();
    // near heap: re-inserted from the spill area (keys are relative to this launch's base)
    L.near_n = 0;
    L.nbase = L.now;
    L.nrk = 0; L.nrs = 0;
    for (uint32_t j = 0; j < near_n0; ++j) {
        uint4 e = gp(c.near_spill)[(size_t)j * R + r];
        if (L.near_fits(ent_t(e)) || ent_t(e) - L.now < c.horizon) {
            if (L.near_n < TW_NEAR_CAP && (uint64_t)(ent_t(e) - L.nbase) < 0xFFFFFFFFull) {
                L.near_push(ent_t(e), e.w, e.z);
                continue;
            }
        }
        L.push_far(ent_t(e), e.w, e.z);  // the thread's F_NEARQ hint only speeds up throwTo
    }

    if (LP) {
        // delivery records addressed to this node become phantom deliverer
        // threads, inserted in (t, link, payload, src) order so queue seqs are
        // deterministic whatever order the records arrived in
        uint32_t n_in = gp(c.inbox_n)[r];
        if (n_in > c.IB) {
            L.fail(TW_REP_ERR_QUEUE);
            n_in = c.IB;
        }
        uint32_t used = 0;  // bitmask, IB <= 32
        for (uint32_t k = 0; k < n_in && L.status == TW_REP_RUNNING; ++k) {
            int best = -1;
            uint4 ba = make_uint4(0, 0, 0, 0), bb = ba;
            for (uint32_t j = 0; j < n_in; ++j) {
                if (used & (1u << j)) continue;
                const uint4 GAS* q = gp(c.inbox) + ((size_t)j * R + r) * 2;
                uint4 ea = q[0], eb = q[1];
                bool less = best < 0;
                if (!less) {
                    int64_t t1 = ent_t(ea), t2 = ent_t(ba);
                    uint64_t p1 = ((uint64_t)ea.w << 32) | ea.z, p2 = ((uint64_t)ba.w << 32) | ba.z;
                    less = t1 < t2 || (t1 == t2 && (eb.x < bb.x || (eb.x == bb.x && (p1 < p2 || (p1 == p2 && eb.z < bb.z)))));
                }
                if (less) { best = (int)j; ba = ea; bb = eb; }
            }
            used |= 1u << best;
            int64_t ta = ent_t(ba);
            uint32_t s = L.alloc_slot();
            if (s == 0xFFFFFFFFu) break;
            Th ph;
            ph.w0 = ((TW_PC_DELIVER_STUB + 1) & 0xFFFFu) | ((F_STARTED | F_PHANTOM) << 18);
            ph.w1 = c.lp0 + r;
            ph.w2 = 0xFFFFFFFEu;  // never a throwTo target
            ph.w3 = 0;
            ph.f0 = ph.f1 = ph.f2 = ph.w7 = 0;
            ph.r0 = (int64_t)(((uint64_t)ba.w << 32) | ba.z);  // payload
            ph.r1 = bb.x;                                     // link
            ph.r2 = bb.z;                                     // sending node
            ph.r3 = bb.y;                                     // kind
            bool on_chip = L.enqueue(ph, s, ta);
            L.store_rec(s, ph, on_chip ? ST_CACHE : ST_THROUGH);
        }
        gp(c.inbox_n)[r] = 0;
    }

#ifdef TW_PROF_LITE
#pragma unroll
    for (int i = 0; i < 16; ++i) L.lite[i] = 0;
    LITE_T(lk0);
#endif
    uint32_t pending_main = (uint32_t)sc[SC_PENDING_MAIN * R];
    for (uint32_t it = 0; it < budget; ++it) {
        if (L.status != TW_REP_RUNNING) break;
        LITE_T(l0);
#ifdef TW_PROF_LITE
        uint64_t l1 = l0;
        LITE_ACC(4, 1);
#endif
        Th th;
        uint32_t slot;
        bool run = false;
        if (pending_main) {  // runInSandbox main (TimedT.hs:237): runs at t=0, not a pop
            pending_main = 0;
            slot = 0;
            L.load_rec(0, th);
            run = true;
        } else {
            if (L.live == 0) {  // whileM_ notDone
                if (!LP) L.status = TW_REP_DONE;  // an LP may still receive records
                break;
            }
            if (L.d_ev >= ev_room) break;
            // PQ.minView: the min of the near root and the far sources
            if (L.far_dirty) L.far_min();
            bool use_near = L.near_n != 0;
            int64_t t = 0;
            uint32_t sq = 0;
            if (use_near) { t = L.nbase + (int64_t)(L.nrk >> 32); sq = (uint32_t)L.nrk; slot = L.nrs; }
            if (L.fsrc >= 0 && (!use_near || tless(L.fmt, L.fms, t, sq))) {
                use_near = false;
                t = L.fmt; sq = L.fms; slot = L.fmsl;
            } else if (!use_near) {
                break;  // nothing queued (cannot happen while live > 0)
            }
            if (t > t_end) break;
#ifdef TW_PROF_LITE
            LITE_ACC(13, __builtin_amdgcn_s_memtime() - l0);
#endif
            KLITE_WRAP(14, L.load_rec(slot, th));  // issued first: its latency overlaps the queue maintenance
            KLITE_WRAP(15, if (use_near) L.near_pop(); else if (L.fsrc == TW_RUNS) L.far_pop(); else L.run_pop(L.fsrc));
#ifdef TW_PROF_LITE
            l1 = __builtin_amdgcn_s_memtime();
            LITE_ACC(0, l1 - l0);
#endif
            if (th.w3 != sq) continue;  // superseded by a throwTo re-stamp
            LITE_ACC(5, 1);
            // curTime .= timestamp (TimedT.hs:241-247)
            th.w3 = 0;
            --L.live;
            L.now = t;
            if (t - L.nbase > (int64_t)0x7FFFFFFF) L.near_rebase(t);
            // LP phantom = the deliverer's wake, already counted and hashed by the sender
            const bool phantom = LP && (th_flags(th) & F_PHANTOM);
            if (!phantom) {
                L.final_t = LP ? (t > L.final_t ? t : L.final_t) : t;
                ++L.d_ev;
            }
            uint32_t exc = th_exc(th);  // asyncExceptions . at tid <<.= Nothing (:252)
            if (exc) {
                int64_t val = (int64_t)(int32_t)th.w7;
                th_set_exc(th, 0);
                th.w7 = 0;
                L.hash_add(th.w1, term0(t, TW_KIND_EXC | exc));
                if (!(th_flags(th) & (F_STARTED | F_MAIN))) {  // escapes launchTimedT (:252-263)
                    L.status = TW_REP_ABORTED;
                    L.main_exc = exc;
                    L.store_rec(slot, th, ST_THROUGH);
                    break;
                }
                run = L.unwind(th, slot, exc, val);
            } else {
                if (!phantom) L.hash_add(th.w1, term0(t, TW_KIND_RESUME | th_pc(th)));
                run = true;
            }
        }
#ifdef TW_PROF_LITE
        LITE_T(l2);
        LITE_ACC(1, l2 - l1);
#endif
        if (run) L.step(th, slot);
#ifdef TW_PROF_LITE
        LITE_ACC(2, __builtin_amdgcn_s_memtime() - l2);
#endif
    }
#ifdef TW_PROF_LITE
    LITE_ACC(3, __builtin_amdgcn_s_memtime() - lk0);
    if (c.prof)
        for (int i = 0; i < 16; ++i)
            __hip_atomic_fetch_add(gp(c.prof) + i, (unsigned long long)L.lite[i], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
#endif
    L.flush_cache();
    sc[SC_PENDING_MAIN * R] = pending_main;
    if (!LP && L.status == TW_REP_RUNNING && L.live == 0) L.status = TW_REP_DONE;

    sc[SC_NOW * R] = (uint64_t)L.now; sc[SC_FINAL_T * R] = (uint64_t)L.final_t;
    sc[SC_SEQ * R] = L.seq; sc[SC_TIDC * R] = L.tidc; sc[SC_LIVE * R] = L.live;
    sc[SC_NEAR_N * R] = L.near_n; sc[SC_FAR_N * R] = L.far_n;
    sc[SC_STATUS * R] = L.status; sc[SC_MAIN_EXC * R] = L.main_exc;
    sc[SC_FREE_N * R] = L.free_n; sc[SC_FTOP * R] = L.ftop; sc[SC_BUMP * R] = L.bump;
    sc[SC_TMO_CTR * R] = L.tmo_ctr;
    sc[SC_EVENTS * R] = events0 + L.d_ev;
    sc[SC_DELIVERED * R] += L.d_dl; sc[SC_DROPPED * R] += L.d_dr;
    sc[SC_UNDELIV * R] += L.d_ud; sc[SC_THREADS * R] += L.d_th;
#pragma unroll
    for (int j = 0; j < TW_RUNS; ++j) {
        sc[(SC_RH0 + j) * R] = L.rh[j];
        sc[(SC_RC0 + j) * R] = L.rn[j];
    }
    for (uint32_t j = 0; j < L.near_n; ++j) {
        uint64_t k = L.nk[j * TW_WG];
        gp(c.near_spill)[(size_t)j * R + r] = ent(L.nbase + (int64_t)(k >> 32), L.ns[j * TW_WG], (uint32_t)k);
    }
    bool active = L.status == TW_REP_RUNNING && L.d_ev < ev_room;
    int64_t tn = INT64_MAX;
    if (L.far_dirty) L.far_min();
    if (L.near_n) tn = L.nbase + (int64_t)(L.nrk >> 32);
    if (L.fsrc >= 0 && L.fmt < tn) tn = L.fmt;
    if (active && (tn == INT64_MAX || tn > t_end) && !pending_main) active = false;  // parked beyond t_end
    if (LP && L.status == TW_REP_RUNNING && tn != INT64_MAX)
        __hip_atomic_fetch_min(gp(c.next_t), (uint64_t)tn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (active) __hip_atomic_fetch_add(gp(c.n_active), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


// Delivery records -> inboxes of local nodes (or the foreign buffer for the
// host exchange).  One thread per record; the per-node inbox slot is claimed
// with an atomic, and the drain at the next window start sorts them.
__global__ void __launch_bounds__(256) tw_lp_scatter(Dev c, const uint4* recs, uint32_t n, uint4* foreign,
                                                     uint32_t* n_foreign, uint32_t foreign_cap) {
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint4 a = gp(recs)[(size_t)i * 2], b = gp(recs)[(size_t)i * 2 + 1];
    uint32_t dst = b.w;
    if (dst >= c.lp0 && dst < c.lp0 + c.R) {
        uint32_t lp = dst - c.lp0;
        uint32_t k = __hip_atomic_fetch_add(gp(c.inbox_n) + lp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k >= c.IB) {
            __hip_atomic_fetch_or(gp(c.lp_err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        uint4 GAS* q = gp(c.inbox) + ((size_t)k * c.R + lp) * 2;
        q[0] = a;
        q[1] = b;
        int64_t ta = ent_t(a);
        __hip_atomic_fetch_min(gp(c.next_t), (uint64_t)ta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (foreign) {
        uint32_t k = __hip_atomic_fetch_add(gp(n_foreign), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k >= foreign_cap) {
            __hip_atomic_fetch_or(gp(c.lp_err), 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        gp(foreign)[(size_t)k * 2] = a;
        gp(foreign)[(size_t)k * 2 + 1] = b;
    } else {
        __hip_atomic_fetch_or(gp(c.lp_err), 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

}  // namespace

// ======================================================================= C ABI
struct tw_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    Dev d{};
    bool loaded = false;
    std::vector<void*> allocs;
    uint32_t* h_active = nullptr;  // pinned
    uint32_t main_pc = 0, main_node = 0;
    int64_t* main_regs = nullptr;  // device copies for tw_reset
    int64_t* nv_init = nullptr;
    uint32_t* listen_init = nullptr;
    size_t lds_bytes = 0;
    // LP mode
    bool lp = false;
    uint4* foreign = nullptr;      // [out_cap][2]
    uint32_t* n_foreign = nullptr;
    uint4* staging = nullptr;      // inject staging [out_cap][2]
    std::vector<double> launch_ms;
    std::vector<hipEvent_t> ev_pool;
};

namespace {

int hip_fail(hipError_t e) {
    (void)e;
    return TW_ERR_HIP;
}

#define HIPCHK(x)                                     \
    do {                                              \
        hipError_t _e = (x);                          \
        if (_e != hipSuccess) {                       \
            fprintf(stderr, "timewarp: %s failed: %s\n", #x, hipGetErrorString(_e)); \
            return _e == hipErrorOutOfMemory ? TW_ERR_OOM : hip_fail(_e); \
        }                                             \
    } while (0)

template <class T>
int dalloc(tw_ctx* c, T** p, size_t n) {
    void* q = nullptr;
    if (n == 0) n = 1;
    HIPCHK(hipMalloc(&q, n * sizeof(T)));
    c->allocs.push_back(q);
    *p = (T*)q;
    return TW_OK;
}

void free_all(tw_ctx* c) {
    for (void* p : c->allocs) (void)hipFree(p);
    c->allocs.clear();
    c->loaded = false;
}

}  // namespace

extern "C" {

const char* tw_version(void) { return "timewarp-mi355x 0.2 (gfx950, lane-per-replica, near-cap 16, LDS write-back record cache)"; }

const char* tw_strerror(int code) {
    switch (code) {
    case TW_OK: return "ok";
    case TW_ERR_INVALID: return "invalid argument or scenario descriptor";
    case TW_ERR_NO_DEVICE: return "no HIP device";
    case TW_ERR_HIP: return "HIP runtime error";
    case TW_ERR_OOM: return "device out of memory";
    case TW_ERR_STATE: return "call out of order";
    case TW_ERR_REPLICA: return "replica error";
    default: return "unknown error";
    }
}

int tw_create(int device, tw_ctx** out) {
    if (!out) return TW_ERR_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device < 0 || device >= n) return TW_ERR_NO_DEVICE;
    tw_ctx* c = new (std::nothrow) tw_ctx;
    if (!c) return TW_ERR_OOM;
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc((void**)&c->h_active, sizeof(uint32_t)) != hipSuccess) {
        delete c;
        return TW_ERR_HIP;
    }
    *out = c;
    return TW_OK;
}

void tw_destroy(tw_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    free_all(c);
    for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
    if (c->h_active) (void)hipHostFree(c->h_active);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

static int validate(const tw_scenario_desc* s) {
    if (!s || s->abi_version != TW_ABI_VERSION) return TW_ERR_INVALID;
    if (s->n_replicas == 0 || s->n_nodes == 0 || !s->insns || s->n_insns < TW_PC_USER || s->n_insns > 0xFFFF)
        return TW_ERR_INVALID;
    if (s->max_slots < 1 || s->queue_capacity < 1 || s->link_depth < 1 || !s->out_off) return TW_ERR_INVALID;
    if (s->main_pc >= s->n_insns || s->main_node >= s->n_nodes || s->max_timeouts > 65536) return TW_ERR_INVALID;
    if (s->n_links && (!s->link_dst || !s->link_rev)) return TW_ERR_INVALID;
    if (s->n_listener_sets && (!s->listener_pc || !s->n_msg_kinds)) return TW_ERR_INVALID;
    // fixed stubs
    const uint32_t stub_ops[6] = {TW_OP_WAIT_REG, TW_OP_DELIVER, TW_OP_END, TW_OP_WAIT_REG, TW_OP_TMO_FIRE, TW_OP_END};
    for (int i = 0; i < 6; ++i)
        if ((s->insns[i].w0 & 0xFF) != stub_ops[i]) return TW_ERR_INVALID;
    for (uint32_t l = 0; l < s->n_links; ++l)
        if (s->link_dst[l] >= s->n_nodes) return TW_ERR_INVALID;
    if (s->out_off[s->n_nodes] != s->n_links) return TW_ERR_INVALID;
    return TW_OK;
}

int tw_reset(tw_ctx* c);

static int load_common(tw_ctx* c, const tw_scenario_desc* s, bool lp, uint32_t lp_begin, uint32_t lp_count,
                       int64_t lookahead, uint32_t inbox_cap, uint32_t outbox_cap) {
    if (!c) return TW_ERR_INVALID;
    int v = validate(s);
    if (v) return v;
    if (lp && (s->n_replicas != 1 || lp_count == 0 || (uint64_t)lp_begin + lp_count > s->n_nodes ||
               inbox_cap == 0 || inbox_cap > 32 || outbox_cap == 0 || lookahead < 1))
        return TW_ERR_INVALID;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    free_all(c);
    Dev& d = c->d;
    d = Dev{};
    c->lp = lp;
    d.R = lp ? lp_count : s->n_replicas;
    d.S = s->max_slots; d.Q = s->queue_capacity;
    d.N = lp ? 1 : s->n_nodes;  // per-lane node arrays
    d.Ntot = s->n_nodes;
    d.lp0 = lp ? lp_begin : 0;
    d.IB = inbox_cap;
    d.out_cap = outbox_cap;
    d.lookahead = lookahead;
    d.L = s->n_links; d.D = s->link_depth; d.T = s->max_timeouts;
    d.n_insns = s->n_insns; d.n_consts = s->n_consts; d.n_sets = s->n_listener_sets; d.n_kinds = s->n_msg_kinds;
    d.horizon = s->near_horizon_us;
    d.Cr = s->run_capacity;
    const size_t R = d.R;
    const size_t Rt = s->n_replicas;  // replica dimension of the host tables
    c->lds_bytes = fixed_lds_bytes() + 8ull * (d.n_insns + 1) + 8ull * d.n_consts;
    if (c->lds_bytes > 160 * 1024) { free_all(c); return TW_ERR_INVALID; }  // program + constants must fit in LDS
    HIPCHK(hipFuncSetAttribute((const void*)tw_run_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)c->lds_bytes));
    HIPCHK(hipFuncSetAttribute((const void*)tw_run_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)c->lds_bytes));
    int e;
#define ALLOC(p, n) if ((e = dalloc(c, &p, (n))) != TW_OK) { free_all(c); return e; }
    uint2* insns; int64_t* consts; uint32_t *lpc, *out_off, *ldst, *lrev, *ltab = nullptr;
    ALLOC(insns, (size_t)d.n_insns + 1);  // +1 NOP: the fall-through prefetch may read one past
    ALLOC(consts, d.n_consts);
    ALLOC(lpc, (size_t)d.n_sets * d.n_kinds);
    ALLOC(out_off, (size_t)d.Ntot + 1);
    ALLOC(ldst, d.L);
    ALLOC(lrev, d.L);
    if (s->link_table) ALLOC(ltab, (size_t)d.L * d.D * Rt);
    ALLOC(d.scal, (size_t)SC_COUNT * R);
    ALLOC(d.slots, (size_t)d.S * R * 4);
    ALLOC(d.free_stk, (size_t)d.S * R);
    ALLOC(d.far, (size_t)d.Q * R);
    ALLOC(d.runs, (size_t)(d.Cr ? TW_RUNS * (size_t)d.Cr : 1) * R);
    ALLOC(d.near_spill, (size_t)TW_NEAR_CAP * R);
    ALLOC(d.nvars, (size_t)d.N * 4 * R);
    ALLOC(d.hash, (size_t)d.N * R);
    ALLOC(d.bind, (size_t)d.N * R);
    ALLOC(d.bind_own, (size_t)d.N * R);
    ALLOC(d.link_ord, (size_t)(d.L ? d.L : 1) * (lp ? 1 : R));
    ALLOC(d.tmo_done, (size_t)(d.T ? d.T : 1) * R);
    ALLOC(d.n_active, 1);
#ifdef TW_PROF_LITE
    ALLOC(d.prof, P_COUNT);
    HIPCHK(hipMemsetAsync(d.prof, 0, 8 * P_COUNT, c->stream));
#endif
    if (lp) {
        ALLOC(d.hash_g, (size_t)d.Ntot);
        ALLOC(d.inbox, (size_t)d.IB * R * 2);
        ALLOC(d.inbox_n, R);
        ALLOC(d.outbox, (size_t)d.out_cap * 2);
        ALLOC(d.out_n, 1);
        ALLOC(d.next_t, 1);
        ALLOC(d.lp_err, 1);
        ALLOC(c->foreign, (size_t)d.out_cap * 2);
        ALLOC(c->n_foreign, 1);
        ALLOC(c->staging, (size_t)d.out_cap * 2);
    }
    int64_t *mregs = nullptr, *nvi = nullptr;
    if (s->main_regs && !lp) ALLOC(mregs, R * 4);
    if (s->node_vars) ALLOC(nvi, (size_t)d.Ntot * 4);
    uint32_t* lsi = nullptr;
    if (s->node_listen) ALLOC(lsi, (size_t)d.Ntot);
#undef ALLOC
    hipStream_t st = c->stream;
    HIPCHK(hipMemsetAsync(insns, 0, sizeof(tw_insn) * (d.n_insns + 1), st));
    HIPCHK(hipMemcpyAsync(insns, s->insns, sizeof(tw_insn) * d.n_insns, hipMemcpyHostToDevice, st));
    if (d.n_consts) HIPCHK(hipMemcpyAsync(consts, s->consts, 8 * d.n_consts, hipMemcpyHostToDevice, st));
    if (d.n_sets) HIPCHK(hipMemcpyAsync(lpc, s->listener_pc, 4ull * d.n_sets * d.n_kinds, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(out_off, s->out_off, 4ull * (d.Ntot + 1), hipMemcpyHostToDevice, st));
    if (d.L) {
        HIPCHK(hipMemcpyAsync(ldst, s->link_dst, 4ull * d.L, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(lrev, s->link_rev, 4ull * d.L, hipMemcpyHostToDevice, st));
    }
    if (ltab) HIPCHK(hipMemcpyAsync(ltab, s->link_table, 4ull * d.L * d.D * Rt, hipMemcpyHostToDevice, st));
    if (mregs) HIPCHK(hipMemcpyAsync(mregs, s->main_regs, 32ull * R, hipMemcpyHostToDevice, st));
    if (nvi) HIPCHK(hipMemcpyAsync(nvi, s->node_vars, 32ull * d.Ntot, hipMemcpyHostToDevice, st));
    if (lsi) HIPCHK(hipMemcpyAsync(lsi, s->node_listen, 4ull * d.Ntot, hipMemcpyHostToDevice, st));
    d.insns = insns; d.consts = consts; d.lpc = lpc; d.out_off = out_off; d.link_dst = ldst; d.link_rev = lrev;
    d.link_table = ltab;
    c->main_pc = s->main_pc;
    c->main_node = s->main_node;
    c->main_regs = mregs;
    c->nv_init = nvi;
    c->listen_init = lsi;
    c->loaded = true;
    int rc = tw_reset(c);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(st));
    return TW_OK;
}

int tw_load(tw_ctx* c, const tw_scenario_desc* s) { return load_common(c, s, false, 0, 0, 0, 0, 0); }

int tw_lp_load(tw_ctx* c, const tw_scenario_desc* s, uint32_t lp_begin, uint32_t lp_count, int64_t lookahead_us,
               uint32_t inbox_cap, uint32_t outbox_cap) {
    return load_common(c, s, true, lp_begin, lp_count, lookahead_us, inbox_cap, outbox_cap);
}

int tw_reset(tw_ctx* c) {
    if (!c) return TW_ERR_INVALID;
    if (!c->loaded) return TW_ERR_STATE;
    HIPCHK(hipSetDevice(c->device));
    const Dev& d = c->d;
    const size_t R = d.R;
    hipStream_t st = c->stream;
    HIPCHK(hipMemsetAsync(d.nvars, 0, 32ull * d.N * R, st));
    HIPCHK(hipMemsetAsync(d.hash, 0, 8ull * d.N * R, st));
    HIPCHK(hipMemsetAsync(d.bind, 0, 4ull * d.N * R, st));
    HIPCHK(hipMemsetAsync(d.link_ord, 0, 4ull * (d.L ? d.L : 1) * (c->lp ? 1 : R), st));
    HIPCHK(hipMemsetAsync(d.tmo_done, 0, (size_t)(d.T ? d.T : 1) * R, st));
    if (c->lp) {
        HIPCHK(hipMemsetAsync(d.hash_g, 0, 8ull * d.Ntot, st));
        HIPCHK(hipMemsetAsync(d.out_n, 0, 4, st));
        HIPCHK(hipMemsetAsync(d.lp_err, 0, 4, st));
        HIPCHK(hipMemsetAsync(c->n_foreign, 0, 4, st));
    }
    uint32_t blocks = (uint32_t)((R + TW_WG - 1) / TW_WG);
    hipLaunchKernelGGL(tw_init_kernel, dim3(blocks), dim3(TW_WG), 0, st, d, c->main_pc, c->main_node,
                       (const int64_t*)c->main_regs, (const int64_t*)c->nv_init, (const uint32_t*)c->listen_init,
                       c->lp ? 1 : 0);
    HIPCHK(hipGetLastError());
    return TW_OK;
}


int tw_run(tw_ctx* c, int64_t t_end_us, uint64_t max_events, tw_stats* out) {
    if (!c) return TW_ERR_INVALID;
    if (!c->loaded) return TW_ERR_STATE;
    auto w0 = std::chrono::steady_clock::now();
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    const Dev& d = c->d;
    uint32_t blocks = (d.R + TW_WG - 1) / TW_WG;
    // events before this call (to report per-call deltas)
    std::vector<uint64_t> ev0(d.R);
    HIPCHK(hipMemcpyAsync(ev0.data(), d.scal + (size_t)SC_EVENTS * d.R, 8ull * d.R, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const uint64_t limit = max_events;  // cumulative per-replica cap
    c->launch_ms.clear();
    const uint32_t budget = 1u << 14;  // pops per lane per launch: bounded kernel time
    const int per_check = 4;           // launches between host checks
    uint32_t launches = 0;
    double kms = 0.0;
    for (int round = 0; round < (1 << 20); ++round) {
        size_t need = 2 * per_check;
        while (c->ev_pool.size() < need) {
            hipEvent_t e;
            HIPCHK(hipEventCreate(&e));
            c->ev_pool.push_back(e);
        }
        for (int i = 0; i < per_check; ++i) {
            HIPCHK(hipMemsetAsync(d.n_active, 0, 4, st));
            if (c->lp) HIPCHK(hipMemsetAsync(d.next_t, 0xFF, 8, st));
            HIPCHK(hipEventRecord(c->ev_pool[2 * i], st));
            if (c->lp)
                hipLaunchKernelGGL(tw_run_kernel<true>, dim3(blocks), dim3(TW_WG), c->lds_bytes, st, d, t_end_us,
                                   limit, budget);
            else
                hipLaunchKernelGGL(tw_run_kernel<false>, dim3(blocks), dim3(TW_WG), c->lds_bytes, st, d, t_end_us,
                                   limit, budget);
            HIPCHK(hipGetLastError());
            HIPCHK(hipEventRecord(c->ev_pool[2 * i + 1], st));
            ++launches;
        }
        HIPCHK(hipMemcpyAsync(c->h_active, d.n_active, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        for (int i = 0; i < per_check; ++i) {
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, c->ev_pool[2 * i], c->ev_pool[2 * i + 1]));
            c->launch_ms.push_back(ms);
            kms += ms;
        }
        if (*c->h_active == 0) break;
    }
    if (out) {
        std::memset(out, 0, sizeof(*out));
        std::vector<tw_replica_result> rr(d.R);
        int rc = tw_read_results(c, rr.data(), d.R);
        if (rc) return rc;
        for (uint32_t i = 0; i < d.R; ++i) {
            out->events += rr[i].events - ev0[i];
            out->delivered += rr[i].delivered;
            out->dropped += rr[i].dropped;
            out->undeliverable += rr[i].undeliverable;
            if (rr[i].final_t > out->max_final_t) out->max_final_t = rr[i].final_t;
            if (rr[i].status == TW_REP_DONE) ++out->replicas_done;
            if (rr[i].status >= TW_REP_ERR_SLOTS) ++out->replicas_error;
        }
        out->sends = out->delivered + out->dropped + out->undeliverable;
        out->launches = launches;
        out->kernel_ms = kms;
        out->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
    }
    return TW_OK;
}

int tw_read_results(tw_ctx* c, tw_replica_result* out, size_t n) {
    if (!c || !out) return TW_ERR_INVALID;
    if (!c->loaded) return TW_ERR_STATE;
    const Dev& d = c->d;
    if (n < d.R) return TW_ERR_INVALID;
    HIPCHK(hipSetDevice(c->device));
    std::vector<uint64_t> sc((size_t)SC_COUNT * d.R);
    HIPCHK(hipMemcpyAsync(sc.data(), d.scal, 8ull * SC_COUNT * d.R, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    auto F = [&](int f, uint32_t i) { return sc[(size_t)f * d.R + i]; };
    for (uint32_t i = 0; i < d.R; ++i) {
        out[i].final_t = (int64_t)F(SC_FINAL_T, i); out[i].events = F(SC_EVENTS, i);
        out[i].delivered = F(SC_DELIVERED, i); out[i].dropped = F(SC_DROPPED, i);
        out[i].undeliverable = F(SC_UNDELIV, i); out[i].status = (uint32_t)F(SC_STATUS, i);
        out[i].main_exc = (uint32_t)F(SC_MAIN_EXC, i); out[i].threads = F(SC_THREADS, i);
    }
    return TW_OK;
}

int tw_read_hashes(tw_ctx* c, uint64_t* out, size_t n) {
    if (!c || !out) return TW_ERR_INVALID;
    if (!c->loaded) return TW_ERR_STATE;
    const Dev& d = c->d;
    if (n < (size_t)d.R * d.N) return TW_ERR_INVALID;
    HIPCHK(hipSetDevice(c->device));
    std::vector<uint64_t> tmp((size_t)d.R * d.N);  // device layout [node][replica]
    HIPCHK(hipMemcpyAsync(tmp.data(), d.hash, 8ull * d.R * d.N, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (uint32_t node = 0; node < d.N; ++node)
        for (uint32_t r = 0; r < d.R; ++r) out[(size_t)r * d.N + node] = tmp[(size_t)node * d.R + r];
    return TW_OK;
}

int tw_read_final(tw_ctx* c, int64_t* max_final_t, uint64_t* delivered, uint64_t* dropped, uint64_t* events) {
    if (!c) return TW_ERR_INVALID;
    if (!c->loaded) return TW_ERR_STATE;
    std::vector<tw_replica_result> rr(c->d.R);
    int rc = tw_read_results(c, rr.data(), rr.size());
    if (rc) return rc;
    int64_t ft = 0;
    uint64_t dl = 0, dr = 0, ev = 0;
    for (auto& x : rr) {
        ft = x.final_t > ft ? x.final_t : ft;
        dl += x.delivered; dr += x.dropped; ev += x.events;
    }
    if (max_final_t) *max_final_t = ft;
    if (delivered) *delivered = dl;
    if (dropped) *dropped = dr;
    if (events) *events = ev;
    return TW_OK;
}

static int lp_scatter(tw_ctx* c, const uint4* recs, uint32_t n, bool to_foreign) {
    const Dev& d = c->d;
    if (n == 0) return TW_OK;
    uint32_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(tw_lp_scatter, dim3(blocks), dim3(256), 0, c->stream, d, recs, n,
                       to_foreign ? c->foreign : nullptr, c->n_foreign, d.out_cap);
    HIPCHK(hipGetLastError());
    return TW_OK;
}

int tw_lp_window(tw_ctx* c, int64_t t_end_excl, int64_t* next_t, uint64_t* n_foreign) {
    if (!c || !next_t) return TW_ERR_INVALID;
    if (!c->loaded || !c->lp) return TW_ERR_STATE;
    tw_stats st{};
    int rc = tw_run(c, t_end_excl - 1, UINT64_MAX, nullptr);
    if (rc) return rc;
    (void)st;
    const Dev& d = c->d;
    hipStream_t s = c->stream;
    uint32_t nout = 0;
    HIPCHK(hipMemcpyAsync(&nout, d.out_n, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (nout > d.out_cap) nout = d.out_cap;
    rc = lp_scatter(c, d.outbox, nout, true);
    if (rc) return rc;
    HIPCHK(hipMemsetAsync(d.out_n, 0, 4, s));
    uint64_t nt = 0;
    uint32_t nf = 0, err = 0;
    HIPCHK(hipMemcpyAsync(&nt, d.next_t, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&nf, c->n_foreign, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&err, d.lp_err, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (err) return TW_ERR_REPLICA;
    *next_t = nt > (uint64_t)INT64_MAX ? INT64_MAX : (int64_t)nt;
    if (n_foreign) *n_foreign = nf;
    return TW_OK;
}

int tw_lp_take_outbox(tw_ctx* c, tw_lp_record* out, size_t cap, size_t* n) {
    if (!c || !n) return TW_ERR_INVALID;
    if (!c->loaded || !c->lp) return TW_ERR_STATE;
    hipStream_t s = c->stream;
    uint32_t nf = 0;
    HIPCHK(hipMemcpyAsync(&nf, c->n_foreign, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (nf > cap || !out) { *n = nf; return nf > cap ? TW_ERR_INVALID : TW_OK; }
    if (nf) HIPCHK(hipMemcpyAsync(out, c->foreign, 32ull * nf, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemsetAsync(c->n_foreign, 0, 4, s));
    HIPCHK(hipStreamSynchronize(s));
    *n = nf;
    return TW_OK;
}

int tw_lp_inject(tw_ctx* c, const tw_lp_record* recs, size_t n, int64_t* next_t) {
    if (!c || (n && !recs)) return TW_ERR_INVALID;
    if (!c->loaded || !c->lp) return TW_ERR_STATE;
    const Dev& d = c->d;
    if (n > d.out_cap) return TW_ERR_INVALID;
    hipStream_t s = c->stream;
    if (n) {
        HIPCHK(hipMemcpyAsync(c->staging, recs, 32ull * n, hipMemcpyHostToDevice, s));
        int rc = lp_scatter(c, c->staging, (uint32_t)n, false);
        if (rc) return rc;
    }
    uint64_t nt = 0;
    uint32_t err = 0;
    HIPCHK(hipMemcpyAsync(&nt, d.next_t, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&err, d.lp_err, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (err) return TW_ERR_REPLICA;
    if (next_t) *next_t = nt > (uint64_t)INT64_MAX ? INT64_MAX : (int64_t)nt;
    return TW_OK;
}

int tw_lp_results(tw_ctx* c, tw_replica_result* agg, uint64_t* node_hashes, size_t n_nodes) {
    if (!c || !agg) return TW_ERR_INVALID;
    if (!c->loaded || !c->lp) return TW_ERR_STATE;
    const Dev& d = c->d;
    std::vector<tw_replica_result> rr(d.R);
    int rc = tw_read_results(c, rr.data(), rr.size());
    if (rc) return rc;
    std::memset(agg, 0, sizeof(*agg));
    agg->status = TW_REP_DONE;
    for (auto& x : rr) {
        agg->final_t = x.final_t > agg->final_t ? x.final_t : agg->final_t;
        agg->events += x.events; agg->delivered += x.delivered; agg->dropped += x.dropped;
        agg->undeliverable += x.undeliverable; agg->threads += x.threads;
        if (x.main_exc) agg->main_exc = x.main_exc;
        if (x.status >= TW_REP_ABORTED) agg->status = x.status;
    }
    if (node_hashes) {
        if (n_nodes < d.Ntot) return TW_ERR_INVALID;
        HIPCHK(hipMemcpyAsync(node_hashes, d.hash_g, 8ull * d.Ntot, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    return TW_OK;
}

#ifdef TW_PROF_LITE
// Diagnostic build only: copy the P_COUNT counters out, optionally zeroing them.
int tw_prof_read(tw_ctx* c, unsigned long long* out, size_t cap, int reset) {
    if (!c || !out || !c->loaded || !c->d.prof) return TW_ERR_STATE;
    size_t n = cap < (size_t)P_COUNT ? cap : (size_t)P_COUNT;
    HIPCHK(hipMemcpy(out, c->d.prof, 8 * n, hipMemcpyDeviceToHost));
    if (reset) HIPCHK(hipMemset(c->d.prof, 0, 8 * P_COUNT));
    return (int)n;
}
#endif

int tw_last_launch_ms(tw_ctx* c, double* out, size_t cap) {
    if (!c || !out) return TW_ERR_INVALID;
    size_t n = c->launch_ms.size() < cap ? c->launch_ms.size() : cap;
    for (size_t i = 0; i < n; ++i) out[i] = c->launch_ms[i];
    return (int)n;
}

}  // extern "C"
