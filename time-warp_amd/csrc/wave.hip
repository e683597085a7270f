// wave.hip — the wave-per-replica event kernel (geometry TW_GEO_WAVE) of
// libtimewarp.so, for batches with few replicas per GPU (BASELINE config 5,
// 4,096 replicas; config 3 sharded over 8 GPUs, 8,192 per GPU).
//
// Replaces, for one replica per wavefront, the same pure-emulation runner as
// engine.hip:
//   launchTimedT / runTimedT   src/Control/TimeWarp/Timed/TimedT.hs:234-304
//   fork / wait / throwTo / timeout               TimedT.hs:326-376
// with the emulated transfer of SURVEY.md Appendix A.3.  Results are
// bit-identical to the lane-per-replica kernels and to the oracle's canonical
// (t, seq) order.
//
// Mapping.  A replica's TimedT loop is sequential (one pop at
// a time, TimedT.hs:239-263); with few replicas, lane-per-replica leaves the
// chip empty and each lane's events form a chain of dependent memory round
// trips.  Here a whole wavefront serves one replica:
//   * the control state (clock, counters, the running thread's record and
//     registers) is wave-uniform -- scalar registers and uniform branches;
//   * the pending-event queue's near tier lives in VECTOR registers: each of
//     the 64 lanes holds K entries (a 64-bit (t, seq) key + a slot), so the
//     queue holds 64*K events on chip with no LDS or memory latency.  A pop is
//     a DPP min-reduction over the lanes' cached local minima
//     (row_shr prefix-min + 4 readlanes) and a K-entry rescan in the winning
//     lane; a push is a ballot over the lanes with room;
//   * events beyond the near horizon go to monotone FIFO runs and a binary
//     heap in HBM, laid out per replica (one replica's far queue is contiguous);
//   * many replicas per SIMD (up to 8 waves) hide the remaining HBM latency of
//     thread records and node state.
#include <cstdlib>

#include "tw_dev.hpp"

#define TW_STEP_CAP (1u << 22)  // instructions per thread step (== oracle kStepCap, engine.hip)

namespace tw {
namespace {

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
    return ((uint64_t)rfl((uint32_t)(v >> 32)) << 32) | rfl((uint32_t)v);
}
__device__ __forceinline__ int64_t rfl64s(int64_t v) { return (int64_t)rfl64((uint64_t)v); }
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
__device__ __forceinline__ uint64_t rdl64(uint64_t v, uint32_t l) {
    return ((uint64_t)rdl((uint32_t)(v >> 32), l) << 32) | rdl((uint32_t)v, l);
}
__device__ __forceinline__ uint32_t dpp_shr(uint32_t v, int n) {
    switch (n) {
    case 1: return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x111, 0xF, 0xF, false);
    case 2: return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x112, 0xF, 0xF, false);
    case 4: return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x114, 0xF, 0xF, false);
    default: return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x118, 0xF, 0xF, false);
    }
}
// min over the 64 lanes of a 64-bit value (wave-uniform result): row prefix-min
// by DPP row_shr 1/2/4/8 (a lane whose source is outside its row keeps its own
// value), then the four row minima by readlane.
__device__ __forceinline__ uint64_t wave_min64(uint64_t v) {
#pragma unroll
    for (int n = 1; n <= 8; n <<= 1) {
        const uint64_t o = ((uint64_t)dpp_shr((uint32_t)(v >> 32), n) << 32) | dpp_shr((uint32_t)v, n);
        v = o < v ? o : v;
    }
    uint64_t m = rdl64(v, 15);
    const uint64_t m1 = rdl64(v, 31), m2 = rdl64(v, 47), m3 = rdl64(v, 63);
    m = m1 < m ? m1 : m;
    m = m2 < m ? m2 : m;
    return m3 < m ? m3 : m;
}

// (branch-free masked stores st32/st128/st8/atom_add64: tw_dev.hpp)
__device__ __forceinline__ void st64(uint64_t GAS* p, uint64_t v, uint64_t mask = 1) {
    uint64_t sv;
    asm volatile("s_mov_b64 %0, exec\n\ts_and_b64 exec, exec, %3\n\tglobal_store_dwordx2 %1, %2, off\n\t"
                 "s_mov_b64 exec, %0" : "=&s"(sv) : "v"(p), "v"(v), "s"(mask) : "memory", "scc");
}
__device__ __forceinline__ void st_i64(int64_t GAS* p, int64_t v) { st64((uint64_t GAS*)p, (uint64_t)v); }

// Read-only tables (program image, constants, topology): constant address
// space, so uniform-address reads become scalar loads.
#if defined(__HIP_DEVICE_COMPILE__)
#define CAS __attribute__((address_space(4)))
#else
#define CAS
#endif
template <class T>
__device__ __forceinline__ const T CAS* cp(const T* p) {
    return (const T CAS*)p;
}

// The running thread's record, wave-uniform (scalar registers).  Registers
// are indexed by uniform selects, never by a dynamic array index (that would
// put them in scratch memory).
struct URec {
    uint32_t w0, w1, w2, w3, f0, f1, xl, xh;
    int64_t r0, r1, r2, r3;
    __device__ __forceinline__ int64_t reg(uint32_t i) const {
        return i == 0 ? r0 : i == 1 ? r1 : i == 2 ? r2 : r3;
    }
    __device__ __forceinline__ void set_reg(uint32_t i, int64_t v) {
        r0 = i == 0 ? v : r0; r1 = i == 1 ? v : r1; r2 = i == 2 ? v : r2; r3 = i == 3 ? v : r3;
    }
};
__device__ __forceinline__ void urec_load(const uint4 GAS* p, uint64_t qs, URec& t) {
    // lanes 0..3 fetch one quad each (records are quad-major: stride qs); readlane to scalars
    const uint4 q = p[(__lane_id() & 3u) * qs];
    t.w0 = rdl(q.x, 0); t.w1 = rdl(q.y, 0); t.w2 = rdl(q.z, 0); t.w3 = rdl(q.w, 0);
    t.f0 = rdl(q.x, 1); t.f1 = rdl(q.y, 1); t.xl = rdl(q.z, 1); t.xh = rdl(q.w, 1);
    t.r0 = (int64_t)(((uint64_t)rdl(q.y, 2) << 32) | rdl(q.x, 2));
    t.r1 = (int64_t)(((uint64_t)rdl(q.w, 2) << 32) | rdl(q.z, 2));
    t.r2 = (int64_t)(((uint64_t)rdl(q.y, 3) << 32) | rdl(q.x, 3));
    t.r3 = (int64_t)(((uint64_t)rdl(q.w, 3) << 32) | rdl(q.z, 3));
}
// store quads [q0, q1) of the record (lanes q0..q1-1, one request)
__device__ __forceinline__ void urec_store(uint4 GAS* p, uint64_t qs, const URec& t, uint32_t q0, uint32_t q1) {
    const uint32_t l = __lane_id() & 3u;
    const bool a = l == 0, b = l == 1, c = l == 2;
    const uint4 q = make_uint4(a ? t.w0 : b ? t.f0 : c ? (uint32_t)t.r0 : (uint32_t)t.r2,
                               a ? t.w1 : b ? t.f1 : c ? (uint32_t)((uint64_t)t.r0 >> 32) : (uint32_t)((uint64_t)t.r2 >> 32),
                               a ? t.w2 : b ? t.xl : c ? (uint32_t)t.r1 : (uint32_t)t.r3,
                               a ? t.w3 : b ? t.xh : c ? (uint32_t)((uint64_t)t.r1 >> 32) : (uint32_t)((uint64_t)t.r3 >> 32));
    st128(p + l * qs, q, ((1ull << q1) - 1) & ~((1ull << q0) - 1));
}
__device__ __forceinline__ uint32_t u_pc(const URec& t) { return t.w0 & 0xFFFFu; }
__device__ __forceinline__ uint32_t u_nfr(const URec& t) { return (t.w0 >> 16) & 15u; }
__device__ __forceinline__ uint32_t u_flags(const URec& t) { return (t.w0 >> FL_SHIFT) & 0x3Fu; }
__device__ __forceinline__ uint32_t u_exc(const URec& t) { return t.w0 >> EXC_SHIFT; }
__device__ __forceinline__ void u_set_pc(URec& t, uint32_t pc) { t.w0 = (t.w0 & 0xFFFF0000u) | (pc & 0xFFFFu); }
__device__ __forceinline__ void u_set_nfr(URec& t, uint32_t n) { t.w0 = (t.w0 & ~(15u << 16)) | (n << 16); }
__device__ __forceinline__ void u_set_exc(URec& t, uint32_t c) {
    t.w0 = (t.w0 & ((1u << EXC_SHIFT) - 1u)) | (c << EXC_SHIFT);
}

enum { W_NONE, W_YIELD, W_SPAWN, W_EXIT, W_STOP, W_DIED };

// Cold per-replica state in LDS (one workgroup = one wave = one replica):
// the far runs' bookkeeping, the far heap's top and the rarely-bumped
// counters.  Keeping them out of scalar registers leaves the event loop's
// uniform state within the SGPR file.
struct WCold {
    int64_t rh_t[TW_RUNS], rt_t[TW_RUNS];           // run head / tail time
    uint32_t rh_s[TW_RUNS], rh_sl[TW_RUNS], rt_s[TW_RUNS], rn[TW_RUNS], ri[TW_RUNS];
    int64_t fh_t;                                    // far heap top
    uint32_t fh_s, fh_sl;
    uint32_t dl, dr, ud, d_th, main_exc, tmo, trn;   // delivered/dropped/undeliverable, threads, ...
};

// pqueue mode (TW_TIE_PQUEUE): the queue header in LDS while the replica runs
// (loaded from / stored to Dev::pq_hdr around each launch, PQ_* words)
struct PQCold {
    uint32_t n, nfree, bump, flen;  // size, free-node stack depth, nodes ever used, forest length
    uint4 min;                      // MinQueue's held minimum {t lo, t hi, slot, seq}
    uint32_t forest[32];            // root node of rank k, or PQ_NONE (a Skip)
};
#define PQ_NONE 0xFFFFFFFFu

// BinaryP transmission time (== tx_us of tw_dev.hpp, context in constant memory)
__device__ __forceinline__ int64_t tx_us_w(const Dev CAS* dv, uint64_t link, uint32_t kind) {
    if (!dv->msg_bytes || !dv->link_bw || kind >= dv->n_kinds) return 0;
    const uint64_t bw = cp(dv->link_bw)[link];
    if (!bw) return 0;
    return (int64_t)(((uint64_t)cp(dv->msg_bytes)[kind] * 1000000ull + bw - 1) / bw);
}

// One replica on one wavefront.  K = near-queue entries per lane (64*K total).
template <int K>
struct Wave {
    const Dev CAS* dv;  // the device context, read through the scalar cache on use
    uint32_t r;      // replica
    uint32_t lane;
    // near queue (per lane, registers): key = (t - nbase) << 32 | seq key; ~0 = free
    uint64_t nk[K];
    uint32_t ns[K];
    uint64_t lmk;    // this lane's minimum key
    uint32_t lmj;    // ... and its entry index
    uint32_t lcnt;   // entries held by this lane
    // wave-uniform state
    uint64_t gmin;   // minimum near key (~0: near queue empty)
    uint32_t near_n, rot;
    int64_t nbase;
    uint32_t far_n;  // binary far heap size (per replica, contiguous in HBM)
    WCold LAS* cw;   // cold state (LDS)
    // the far minimum (over the runs' heads and the heap top), recomputed when dirty
    int64_t fm_t;
    uint32_t fm_s, fm_sl;
    int fm_src;      // -1 none, 0..3 run, TW_RUNS heap
    bool far_dirty;
    // replica scalars
    int64_t now, final_t;
    uint32_t seq, tidc, live, status, free_n, ftop, bump;
    uint32_t d_ev;
    uint64_t hacc;
    uint32_t hnode;

    __device__ Wave(const Dev CAS* d_, uint32_t r_) : dv(d_), r(r_), lane(__lane_id()) {}

    __device__ __forceinline__ size_t ix(size_t i) const { return i * dv->R + r; }
    __device__ __forceinline__ void fail(uint32_t st) {
        if (status == TW_REP_RUNNING) status = st;
    }
    __device__ __forceinline__ uint32_t next_seq() {
        if (seq == 0xFFFFFFFFu) fail(TW_REP_ERR_COUNTER);
        else ++seq;
        return dv->tie_mode ? seq_key(dv->tie_mode, seq) : seq;
    }

    // ------------------------------------------------------ near queue (VGPRs)
    __device__ __forceinline__ void near_init() {
#pragma unroll
        for (int j = 0; j < K; ++j) { nk[j] = ~0ull; ns[j] = 0; }
        lmk = ~0ull; lmj = 0; lcnt = 0;
        gmin = ~0ull; near_n = 0; rot = 0;
    }
    __device__ __forceinline__ void lane_rescan() {
        uint64_t m = ~0ull;
        uint32_t mj = 0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const bool b = nk[j] < m;
            m = b ? nk[j] : m;
            mj = b ? (uint32_t)j : mj;
        }
        lmk = m; lmj = mj;
    }
    __device__ __forceinline__ bool near_fits(int64_t t) const {
        return near_n < 64u * K && t - now < dv->horizon && (uint64_t)(t - nbase) < 0xFFFFFFFFull;
    }
    // push (t, sq, slot): a lane with room (rotating start) takes it
    __device__ __forceinline__ void near_push(int64_t t, uint32_t sq, uint32_t slot) {
        const uint64_t key = ((uint64_t)(t - nbase) << 32) | sq;
        uint64_t room = __builtin_amdgcn_ballot_w64(lcnt < (uint32_t)K);
        if (room == 0) {
            // the lanes' counts disagree with near_n (near_fits let the push
            // through): a broken invariant, reported as a queue error status
            // instead of an entry silently dropped (ctz of an empty ballot)
            fail(TW_REP_ERR_QUEUE);
            return;
        }
        room = (room >> rot) | (rot ? room << (64 - rot) : 0ull);  // rotate right by rot
        const uint32_t tl = (rfl((uint32_t)__builtin_ctzll(room)) + rot) & 63u;
        rot = (tl + 1) & 63u;
        const bool me = lane == tl;  // (selects, not a branch: see st32)
        bool done = !me;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const bool take = !done && nk[j] == ~0ull;
            nk[j] = take ? key : nk[j];
            ns[j] = take ? slot : ns[j];
            lmj = (take && key < lmk) ? (uint32_t)j : lmj;
            done = done || take;
        }
        lmk = (me && key < lmk) ? key : lmk;
        lcnt += me ? 1u : 0u;
        ++near_n;
        gmin = key < gmin ? key : gmin;
    }
    // remove the minimum (key gmin); returns its slot
    __device__ __forceinline__ uint32_t near_pop() {
        const uint64_t hold = __builtin_amdgcn_ballot_w64(lmk == gmin);
        if (hold == 0) {  // no lane holds the minimum: a broken invariant, a status (the caller stops)
            fail(TW_REP_ERR_QUEUE);
            return 0;
        }
        const uint32_t wl = rfl((uint32_t)__builtin_ctzll(hold));
        uint32_t s = 0;
        const bool me = lane == wl;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const bool hit = me && (uint32_t)j == lmj;
            s = hit ? ns[j] : s;
            nk[j] = hit ? ~0ull : nk[j];
        }
        lcnt -= me ? 1u : 0u;
        lane_rescan();
        --near_n;
        gmin = near_n ? wave_min64(lmk) : ~0ull;
        return rdl(s, wl);
    }
    // re-key a queued near entry (seq key old_sq) to (t, sq): throwTo's re-stamp
    __device__ __forceinline__ bool near_rekey(uint32_t old_sq, int64_t t, uint32_t sq, uint32_t slot) {
        bool hit = false;
#pragma unroll
        for (int j = 0; j < K; ++j) hit = hit || (nk[j] != ~0ull && (uint32_t)nk[j] == old_sq);
        const uint64_t m = __builtin_amdgcn_ballot_w64(hit);
        if (!m) return false;
        const uint32_t hl = rfl((uint32_t)__builtin_ctzll(m));
        const bool me = lane == hl;
#pragma unroll
        for (int j = 0; j < K; ++j) nk[j] = (me && nk[j] != ~0ull && (uint32_t)nk[j] == old_sq) ? ~0ull : nk[j];
        lcnt -= me ? 1u : 0u;
        lane_rescan();
        --near_n;
        gmin = near_n ? wave_min64(lmk) : ~0ull;
        near_push(t, sq, slot);
        return true;
    }
    __device__ void near_rebase(int64_t nb) {
        const uint64_t d = (uint64_t)(nb - nbase) << 32;
#pragma unroll
        for (int j = 0; j < K; ++j) nk[j] = nk[j] == ~0ull ? nk[j] : nk[j] - d;
        lmk = lmk == ~0ull ? lmk : lmk - d;
        gmin = gmin == ~0ull ? gmin : gmin - d;
        nbase = nb;
    }

    // ------------------------------------------ far tier (HBM, per replica)
    // binary heap of {t lo, t hi, slot, seq} at far[r * Q + i]; lane 0 walks it
    __device__ __forceinline__ uint4 GAS* farp(uint32_t i) const { return gp(dv->far) + (size_t)r * dv->Q + i; }
    __device__ __forceinline__ uint4 far_ld(uint32_t i) const {
        const uint4 e = *farp(i);
        return make_uint4(rfl(e.x), rfl(e.y), rfl(e.z), rfl(e.w));
    }
    __device__ __forceinline__ void far_st(uint32_t i, uint4 e) const {
        st128(farp(i), e);
    }
    __device__ __forceinline__ void set_fh(uint4 e) {
        cw->fh_t = ent_t(e); cw->fh_s = e.w; cw->fh_sl = e.z;
        far_dirty = true;
    }
    __device__ void heap_push(int64_t t, uint32_t sq, uint32_t slot) {
        if (far_n >= dv->Q) { fail(TW_REP_ERR_QUEUE); return; }
        far_dirty = true;
        uint32_t i = far_n++;
        while (i > 0) {
            const uint32_t p = (i - 1) >> 1;
            const uint4 q = far_ld(p);
            if (!tless(t, sq, ent_t(q), q.w)) break;
            far_st(i, q);
            i = p;
        }
        const uint4 e = ent(t, slot, sq);
        far_st(i, e);
        if (i == 0) set_fh(e);
    }
    __device__ void heap_pop() {
        const uint32_t n = --far_n;
        far_dirty = true;
        if (n == 0) return;
        const uint4 le = far_ld(n);
        const int64_t t = ent_t(le);
        uint32_t i = 0;
        for (;;) {
            uint32_t ch = 2 * i + 1;
            if (ch >= n) break;
            uint4 b = far_ld(ch);
            if (ch + 1 < n) {
                const uint4 b2 = far_ld(ch + 1);
                if (tless(ent_t(b2), b2.w, ent_t(b), b.w)) { b = b2; ++ch; }
            }
            if (!tless(ent_t(b), b.w, t, le.w)) break;
            far_st(i, b);
            if (i == 0) set_fh(b);
            i = ch;
        }
        far_st(i, le);
        if (i == 0) set_fh(le);
    }
    // monotone FIFO runs (patience sorting): run j at runs[(r * TW_RUNS + j) * Cr + pos]
    __device__ __forceinline__ uint4 GAS* runp(uint32_t j, uint32_t pos) const {
        return gp(dv->runs) + ((size_t)r * TW_RUNS + j) * dv->Cr + pos;
    }
    // (run arrays are only indexed by unrolled constants: they stay in registers)
    __device__ bool run_push(int64_t t, uint32_t sq, uint32_t slot) {
        const uint32_t Cr = dv->Cr;
        if (Cr == 0) return false;
        int best = -1, empty = -1;
        int64_t bt = 0;
        uint32_t bs = 0;
#pragma unroll
        for (int j = 0; j < TW_RUNS; ++j) {
            const uint32_t n = rfl(cw->rn[j]);
            const int64_t tt = rfl64s(cw->rt_t[j]);
            const uint32_t ts = rfl(cw->rt_s[j]);
            const bool e = n == 0 && empty < 0;
            empty = e ? j : empty;
            const bool ok = n != 0 && n < Cr && !tless(t, sq, tt, ts) && (best < 0 || tless(bt, bs, tt, ts));
            best = ok ? j : best;
            bt = ok ? tt : bt;
            bs = ok ? ts : bs;
        }
        const int j = best >= 0 ? best : empty;
        if (j < 0) return false;
        const uint32_t n = rfl(cw->rn[j]);
        uint32_t pos = rfl(cw->ri[j]) + n;
        if (pos >= Cr) pos -= Cr;
        st128(runp(j, pos), ent(t, slot, sq));
        if (n == 0) { cw->rh_t[j] = t; cw->rh_s[j] = sq; cw->rh_sl[j] = slot; far_dirty = true; }
        cw->rt_t[j] = t; cw->rt_s[j] = sq;
        cw->rn[j] = n + 1;
        return true;
    }
    __device__ void run_pop(int j) {
        const uint32_t Cr = dv->Cr;
        uint32_t h = rfl(cw->ri[j]) + 1;
        h = h == Cr ? 0 : h;
        cw->ri[j] = h;
        const uint32_t n = rfl(cw->rn[j]) - 1;
        cw->rn[j] = n;
        if (n) {
            const uint4 e = *runp(j, h);
            cw->rh_t[j] = (int64_t)(((uint64_t)rfl(e.y) << 32) | rfl(e.x));
            cw->rh_sl[j] = rfl(e.z);
            cw->rh_s[j] = rfl(e.w);
        }
        far_dirty = true;
    }
    // the far minimum (cached): over the runs' heads and the far heap's top
    __device__ __forceinline__ void far_min() {
        far_dirty = false;
        int src = -1;
        int64_t t = 0;
        uint32_t sq = 0, sl = 0;
        if (far_n) { src = TW_RUNS; t = rfl64s(cw->fh_t); sq = rfl(cw->fh_s); sl = rfl(cw->fh_sl); }
#pragma unroll
        for (int j = 0; j < TW_RUNS; ++j) {
            const uint32_t n = rfl(cw->rn[j]);
            const int64_t ht = rfl64s(cw->rh_t[j]);
            const uint32_t hs = rfl(cw->rh_s[j]), hl = rfl(cw->rh_sl[j]);
            const bool b = n && (src < 0 || tless(ht, hs, t, sq));
            src = b ? j : src;
            t = b ? ht : t;
            sq = b ? hs : sq;
            sl = b ? hl : sl;
        }
        fm_src = src; fm_t = t; fm_s = sq; fm_sl = sl;
    }

    // ---------------------------------------- pqueue mode (TW_TIE_PQUEUE)
    // TimedT's queue itself: pqueue-1.3.1.1 `Data.PQueue.Min.MinQueue` of
    // events ordered by timestamp only (TimedT.hs:100-104), restated node by
    // node from the oracle's transcription (oracle/pqueue_min.hpp, SURVEY.md
    // Appendix B; PARITY UNPINNED against pqueue itself): a held minimum plus
    // a binomial forest, joinBin putting t1 on top iff root t1 <= root t2.
    // Wave-uniform scalar code; nodes in HBM (entries in the replica's far
    // area, links {highest-rank child, next lower-rank sibling}).
    bool pqm;        // the tie mode is TW_TIE_PQUEUE
    PQCold LAS* pc;  // queue header (LDS)
    __device__ __forceinline__ uint4 GAS* pqe(uint32_t i) const { return gp(dv->far) + (size_t)r * dv->Q + i; }
    __device__ __forceinline__ uint2 GAS* pql(uint32_t i) const { return gp(dv->pq_link) + (size_t)r * dv->Q + i; }
    __device__ __forceinline__ uint4 pq_ld(uint32_t i) const {
        const uint4 e = *pqe(i);
        return make_uint4(rfl(e.x), rfl(e.y), rfl(e.z), rfl(e.w));
    }
    __device__ __forceinline__ uint2 pq_lk(uint32_t i) const {
        const uint2 l = *pql(i);
        return make_uint2(rfl(l.x), rfl(l.y));
    }
    __device__ __forceinline__ void pq_setlk(uint32_t i, uint32_t child, uint32_t sib) const {
        st64((uint64_t GAS*)pql(i), ((uint64_t)sib << 32) | child);
    }
    __device__ __forceinline__ uint4 pq_min() const {
        return make_uint4(rfl(pc->min.x), rfl(pc->min.y), rfl(pc->min.z), rfl(pc->min.w));
    }
    __device__ uint32_t pq_new(uint4 e) {
        const uint32_t nf = rfl(pc->nfree);
        uint32_t i;
        if (nf) {
            i = rfl(gp(dv->pq_free)[(size_t)r * dv->Q + nf - 1]);
            pc->nfree = nf - 1;
        } else {
            const uint32_t b = rfl(pc->bump);
            if (b >= dv->Q) { fail(TW_REP_ERR_QUEUE); return PQ_NONE; }
            i = b;
            pc->bump = b + 1;
        }
        st128(pqe(i), e);
        pq_setlk(i, PQ_NONE, PQ_NONE);
        return i;
    }
    __device__ void pq_del(uint32_t i) {
        const uint32_t nf = rfl(pc->nfree);
        st32(gp(dv->pq_free) + (size_t)r * dv->Q + nf, i);
        pc->nfree = nf + 1;
    }
    // joinBin: t1 on top iff root t1 <= root t2; the other becomes its
    // highest-rank child
    __device__ uint32_t pq_join(uint32_t t1, uint32_t t2) {
        const bool top1 = ent_t(pq_ld(t1)) <= ent_t(pq_ld(t2));
        const uint32_t top = top1 ? t1 : t2, sub = top1 ? t2 : t1;
        const uint2 lt = pq_lk(top), ls = pq_lk(sub);
        pq_setlk(sub, ls.x, lt.x);
        pq_setlk(top, sub, lt.y);
        return top;
    }
    // incr: binary-counter carry from rank k up
    __device__ void pq_incr(uint32_t t, uint32_t k) {
        for (;;) {
            const uint32_t fl = rfl(pc->flen);
            if (k >= fl) {  // Nil -> Cons t Nil
                pc->forest[fl] = t;
                pc->flen = fl + 1;
                return;
            }
            const uint32_t u = rfl(pc->forest[k]);
            if (u == PQ_NONE) {  // Skip f -> Cons t f
                pc->forest[k] = t;
                return;
            }
            pc->forest[k] = PQ_NONE;  // Cons t' f -> Skip (incr (joinBin t t') f)
            t = pq_join(t, u);
            ++k;
        }
    }
    // insert' le x (MinQueue n x' ts)
    __device__ void pq_insert(uint4 e) {
        const uint32_t n = rfl(pc->n);
        if (n == 0) {
            pc->min = e;
            pc->n = 1;
            return;
        }
        const uint4 m = pq_min();
        uint32_t t;
        if (ent_t(e) <= ent_t(m)) {
            t = pq_new(m);
            pc->min = e;
        } else {
            t = pq_new(e);
        }
        if (t == PQ_NONE) return;
        pq_incr(t, 0);
        pc->n = n + 1;
    }
    // extractHeap: the root a lower rank wins ties with, its children merged
    // back rank by rank (incrExtract / incrExtract')
    __device__ void pq_extract() {
        const uint32_t fl = rfl(pc->flen);
        int m = -1;
        int64_t mt = 0;
        for (int k = (int)fl - 1; k >= 0; --k) {
            const uint32_t t = rfl(pc->forest[k]);
            if (t == PQ_NONE) continue;
            const int64_t tt = ent_t(pq_ld(t));
            if (m < 0 || tt <= mt) { m = k; mt = tt; }
        }
        if (m < 0) { fail(TW_REP_ERR_QUEUE); return; }  // (n > 0 with an empty forest: a broken invariant)
        const uint32_t w = rfl(pc->forest[m]);
        pc->forest[m] = PQ_NONE;
        uint32_t ch = pq_lk(w).x;  // the rank m-1 child, then its lower-rank siblings
        for (int k = m - 1; k >= 0; --k) {
            const uint32_t kc = ch;
            ch = pq_lk(kc).y;
            const uint32_t u = rfl(pc->forest[k]);
            if (u == PQ_NONE) {
                pc->forest[k] = kc;
            } else {
                pc->forest[k] = PQ_NONE;
                pq_incr(pq_join(u, kc), (uint32_t)k + 1);
            }
        }
        uint32_t f2 = rfl(pc->flen);
        while (f2 && rfl(pc->forest[f2 - 1]) == PQ_NONE) --f2;
        pc->flen = f2;
        pc->min = pq_ld(w);
        pq_del(w);
    }
    // minView
    __device__ uint4 pq_pop() {
        const uint4 out = pq_min();
        const uint32_t n = rfl(pc->n) - 1;
        pc->n = n;
        if (n > 0) pq_extract();
        return out;
    }
    // throwTo's rebuild (TimedT.hs:361-368): fromList . map re-stamp . toList,
    // the entry of thread slot `rs` (if any) moved to tnow
    __device__ void pq_rebuild(uint32_t rs, int64_t tnow) {
        uint4 GAS* scr = gp(dv->pq_scr) + (size_t)r * dv->Q;
        uint32_t cnt = 0;
        while (rfl(pc->n) > 0 && status == TW_REP_RUNNING) {  // toList = toAscList
            uint4 e = pq_pop();
            if (e.z == rs) { e.x = (uint32_t)tnow; e.y = (uint32_t)((uint64_t)tnow >> 32); }
            st128(scr + cnt, e);
            ++cnt;
        }
        for (uint32_t i = cnt; i-- > 0;) {  // fromList = foldr insert empty
            const uint4 e = scr[i];
            pq_insert(make_uint4(rfl(e.x), rfl(e.y), rfl(e.z), rfl(e.w)));
        }
    }

    __device__ __forceinline__ bool enqueue(URec& th, uint32_t slot, int64_t t) {
        const uint32_t s = next_seq();
        if (th.w3 == 0) ++live;
        th.w3 = s;
        if (pqm) {
            pq_insert(ent(t, slot, s));
            th.w0 &= ~(F_NEARQ << FL_SHIFT);
            return false;
        }
        if (near_fits(t)) {
            near_push(t, s, slot);
            th.w0 |= F_NEARQ << FL_SHIFT;
            return true;
        }
        if (!run_push(t, s, slot)) heap_push(t, s, slot);
        th.w0 &= ~(F_NEARQ << FL_SHIFT);
        return false;
    }

    // ----------------------------------------------------- thread records
    __device__ __forceinline__ uint4 GAS* hrec(uint32_t slot) const { return gp(dv->slots) + ix(slot); }
    __device__ __forceinline__ uint32_t alloc_slot() {
        if (free_n) {
            const uint32_t s = ftop;
            if (--free_n) ftop = rfl(gp(dv->free_stk)[ix(free_n - 1)]);
            return s;
        }
        if (bump < dv->S) return bump++;
        fail(TW_REP_ERR_SLOTS);
        return 0xFFFFFFFFu;
    }
    __device__ __forceinline__ void free_slot(uint32_t slot) {
        if (free_n) st32(gp(dv->free_stk) + ix(free_n - 1), ftop);
        ftop = slot;
        ++free_n;
    }
    __device__ __forceinline__ void hash_atomic(uint32_t node, uint64_t v) {
        if (v) atom_add64((unsigned long long GAS*)(gp(dv->hash) + ix(node)), v);
    }
    __device__ __forceinline__ void hash_add(uint32_t node, uint64_t v) {
        if (node == hnode) hacc += v;
        else hash_atomic(node, v);
    }
    __device__ __forceinline__ void hash_flush() {
        hash_atomic(hnode, hacc);
        hacc = 0;
    }
    __device__ __forceinline__ uint32_t GAS* fxp(uint32_t slot, uint32_t i) const {
        return (uint32_t GAS*)(gp(dv->fx) + ((size_t)slot * dv->R + r) * dv->FXQ) + (i - 2);
    }
    __device__ __forceinline__ uint32_t frame(const URec& t, uint32_t slot, uint32_t i) const {
        if (i < 2) return i == 0 ? t.f0 : t.f1;
        return rfl(*fxp(slot, i));
    }
    __device__ __forceinline__ void trace_rec(uint32_t node, int32_t tag, int64_t val) {
        const uint32_t n = rfl(cw->trn);
        cw->trn = n + 1;
        if (n < dv->trace_cap) {
            uint4 GAS* q = gp(dv->trace) + ((size_t)n * dv->R + r) * 2;
            const bool l0 = (lane & 1u) == 0;
            st128(q + (lane & 1u), l0 ? make_uint4((uint32_t)now, (uint32_t)((uint64_t)now >> 32), node, (uint32_t)tag)
                                      : make_uint4((uint32_t)val, (uint32_t)((uint64_t)val >> 32), 0u, 0u), 3);
        }
    }

    // Thread ends: owned listener released, refs invalidated, slot freed; the
    // header quad is stored by the caller.
    __device__ __forceinline__ void die(URec& th, uint32_t slot) {
        if (u_flags(th) & F_OWNS) st32(gp(dv->bind_rel) + ix(th.w1), th.w2);
        th.w2 = 0xFFFFFFFFu;
        th.w3 = 0;
        free_slot(slot);
    }
    // Raise `code` in the running thread (TimedT.hs:183-204): innermost frame
    // first; finally frames set their timeout's done flag (TimedT.hs:376).
    __device__ bool unwind(URec& th, uint32_t slot, uint32_t code, int64_t val) {
        for (int i = (int)u_nfr(th) - 1; i >= 0; --i) {
            const uint32_t f = frame(th, slot, (uint32_t)i);
            const uint32_t mask = f >> 16;
            if (mask == 0) {
                const uint32_t e = f & 0xFFFFu;
                if (e < dv->T) st8(gp(dv->tmo_done) + ix(e), 1);
            } else if (mask & (1u << code)) {
                u_set_nfr(th, (uint32_t)i);
                u_set_pc(th, f & 0xFFFFu);
                th.r0 = val;
                th.r3 = (int64_t)code;
                return true;
            }
        }
        u_set_nfr(th, 0);
        if (u_flags(th) & F_MAIN) cw->main_exc = code;
        die(th, slot);
        urec_store(hrec(slot), dv->RQ, th, 0, 1);
        return false;
    }

    // throwTo (TimedT.hs:357-368): the target's queued event is re-stamped to
    // now with a fresh seq; the first pending exception wins; no yield.
    __device__ void throw_to(URec& self, uint32_t self_slot, int64_t ref, uint32_t code, int64_t val) {
        const uint32_t ts = (uint32_t)ref, tid = (uint32_t)((uint64_t)ref >> 32);
        if (pqm) {
            // TimedT rebuilds its queue on every throwTo, whether or not the
            // target has an event queued (or is alive at all)
            uint32_t rs = PQ_NONE;
            if (ts < dv->S && ts != self_slot) {
                URec t;
                urec_load(hrec(ts), dv->RQ, t);
                if (t.w2 == tid && t.w3 != 0) rs = ts;
            }
            pq_rebuild(rs, now);
        }
        if (ts >= dv->S) return;
        if (ts == self_slot) {
            if (self.w2 != tid) return;
            if (u_exc(self) == 0) { u_set_exc(self, code); self.xl = (uint32_t)val; self.xh = (uint32_t)((uint64_t)val >> 32); }
            return;
        }
        URec t;
        urec_load(hrec(ts), dv->RQ, t);
        if (t.w2 != tid) return;  // dead: the map entry is unobservable
        if (t.w3 != 0 && !pqm) {  // (pqueue mode: re-stamped in place by the rebuild, same seq)
            bool on_chip = (u_flags(t) & F_NEARQ) != 0;
            const uint32_t s = next_seq();
            if (!(on_chip && near_rekey(t.w3, now, s, ts))) {
                on_chip = near_fits(now);
                if (on_chip) near_push(now, s, ts);
                else if (!run_push(now, s, ts)) heap_push(now, s, ts);
            }
            t.w0 = on_chip ? t.w0 | (F_NEARQ << FL_SHIFT) : t.w0 & ~(F_NEARQ << FL_SHIFT);
            t.w3 = s;
        }
        if (u_exc(t) == 0) {
            u_set_exc(t, code);
            t.xl = (uint32_t)val;
            t.xh = (uint32_t)((uint64_t)val >> 32);
        }
        urec_store(hrec(ts), dv->RQ, t, 0, 2);
    }

    // Create a thread queued at now (fork, TimedT.hs:326-339); its record is stored here.
    __device__ bool spawn(uint32_t pc, uint32_t node, int64_t q0, int64_t q1, int64_t q2, int64_t q3, int64_t& ref) {
        const uint32_t s = alloc_slot();
        if (s == 0xFFFFFFFFu) return false;
        if (tidc == 0xFFFFFFFFu) { fail(TW_REP_ERR_COUNTER); return false; }
        const uint32_t tid = tidc++;
        cw->d_th = rfl(cw->d_th) + 1;
        URec ch;
        ch.w0 = pc & 0xFFFFu; ch.w1 = node; ch.w2 = tid; ch.w3 = 0;
        ch.f0 = ch.f1 = ch.xl = ch.xh = 0;
        ch.r0 = q0; ch.r1 = q1; ch.r2 = q2; ch.r3 = q3;
        enqueue(ch, s, now);
        urec_store(hrec(s), dv->RQ, ch, 0, 4);
        ref = (int64_t)(((uint64_t)tid << 32) | s);
        return true;
    }

    // Run the thread's continuation until it yields or ends (TimedT.hs:343-355).
    __device__ void step(URec& th, uint32_t slot) {
        th.w0 |= F_STARTED << FL_SHIFT;
        uint32_t pc = u_pc(th);
        uint32_t fin = W_NONE;
        int64_t yt = 0;
        uint32_t cpc = 0, cnode = 0, cra = 4;
        int64_t q0 = 0, q1 = 0, q2 = 0, q3 = 0;  // the spawned child's registers
        const uint2 CAS* P = cp((const uint2*)dv->insns);
        const int64_t CAS* KP = cp(dv->consts);
        for (uint32_t n = 0;; ++n) {
            if (pc >= dv->n_insns || n >= TW_STEP_CAP) { fail(TW_REP_ERR_INSN); fin = W_STOP; break; }
            const uint2 in = P[pc];
            const uint32_t w = in.x, op = w & 0xFFu, a = (w >> 8) & 3u, b = w >> 16;
            const int32_t imm = (int32_t)in.y;
            const int64_t ra = th.reg(a);
            const int64_t rb = th.reg(b & 3u);
            uint32_t npc = pc + 1;
            bool wr = false;        // the op writes r[a] := wv
            int64_t wv = 0;
            bool thr = false;
            int64_t tref = 0, tval = 0;
            uint32_t tcode = 0;
            switch (op) {
            case TW_OP_NOP: break;
            case TW_OP_END: fin = W_EXIT; break;
            case TW_OP_WAIT_REL: yt = now + KP[imm]; fin = W_YIELD; break;
            case TW_OP_WAIT_ABS: { const int64_t k = KP[imm]; yt = k > now ? k : now; fin = W_YIELD; break; }
            case TW_OP_WAIT_REG: yt = now + (ra > 0 ? ra : 0); fin = W_YIELD; break;
            case TW_OP_FORK: {
                const uint32_t node = b == 0xFFFFu ? th.w1 : (uint32_t)rb;
                if (node >= dv->N) { fail(TW_REP_ERR_INSN); fin = W_STOP; break; }
                cpc = (uint32_t)imm; cnode = node; cra = a;
                q0 = th.r0; q1 = th.r1; q2 = th.r2; q3 = th.r3;
                fin = W_SPAWN;
                break;
            }
            case TW_OP_MYTID: wr = true; wv = (int64_t)(((uint64_t)th.w2 << 32) | slot); break;
            case TW_OP_THROW_TO:
                thr = true; tref = ra; tcode = b & 0xFFu; tval = th.reg((b >> 8) & 3u);
                break;
            case TW_OP_THROW:
                u_set_pc(th, pc + 1);
                if (unwind(th, slot, b & 0xFFu, th.reg((b >> 8) & 3u))) npc = u_pc(th);
                else fin = W_DIED;
                break;
            case TW_OP_CATCH:
            case TW_OP_TMO_PUSH: {
                const uint32_t nf = u_nfr(th);
                if (nf >= dv->max_frames) { fail(TW_REP_ERR_FRAMES); fin = W_STOP; break; }
                const uint32_t fv = op == TW_OP_CATCH ? (b << 16) | ((uint32_t)imm & 0xFFFFu) : (uint32_t)ra & 0xFFFFu;
                if (nf == 0) th.f0 = fv;
                else if (nf == 1) th.f1 = fv;
                else st32(fxp(slot, nf), fv);
                u_set_nfr(th, nf + 1);
                break;
            }
            case TW_OP_UNCATCH: {
                const uint32_t nf = u_nfr(th);
                if (nf == 0 || (frame(th, slot, nf - 1) >> 16) == 0) { fail(TW_REP_ERR_INSN); fin = W_STOP; break; }
                u_set_nfr(th, nf - 1);
                break;
            }
            case TW_OP_SETI: wr = true; wv = imm; break;
            case TW_OP_SETK: wr = true; wv = KP[imm]; break;
            case TW_OP_ADDI: wr = true; wv = ra + imm; break;
            case TW_OP_MULI: wr = true; wv = ra * imm; break;
            case TW_OP_MOV: wr = true; wv = rb; break;
            case TW_OP_ADD: wr = true; wv = ra + rb; break;
            case TW_OP_SUB: wr = true; wv = ra - rb; break;
            case TW_OP_MODI: { const int64_t m = ra % (int64_t)imm; wr = true; wv = m < 0 ? m + imm : m; break; }
            case TW_OP_JMP: npc = (uint32_t)imm; break;
            case TW_OP_JEQ: if (ra == rb) npc = (uint32_t)imm; break;
            case TW_OP_JNE: if (ra != rb) npc = (uint32_t)imm; break;
            case TW_OP_JLT: if (ra < rb) npc = (uint32_t)imm; break;
            case TW_OP_JLE: if (ra <= rb) npc = (uint32_t)imm; break;
            case TW_OP_JEQI: if (ra == (int64_t)(int16_t)b) npc = (uint32_t)imm; break;
            case TW_OP_JNEI: if (ra != (int64_t)(int16_t)b) npc = (uint32_t)imm; break;
            case TW_OP_NOW: wr = true; wv = now; break;
            case TW_OP_NODE: wr = true; wv = th.w1; break;
            case TW_OP_NLOAD: wr = true; wv = rfl64s(gp(dv->nvars)[ix((size_t)th.w1 * 4 + (b & 3u))]); break;
            case TW_OP_NSTORE: st_i64(gp(dv->nvars) + ix((size_t)th.w1 * 4 + (b & 3u)), ra); break;
            case TW_OP_NLOADX:
            case TW_OP_NSTOREX: {
                const uint64_t node = (uint64_t)th.reg((b >> 8) & 3u);
                if (node >= dv->N) { fail(TW_REP_ERR_INSN); fin = W_STOP; break; }
                int64_t GAS* v = &gp(dv->nvars)[ix((size_t)node * 4 + (b & 3u))];
                if (op == TW_OP_NLOADX) { wr = true; wv = rfl64s(*v); }
                else st_i64(v, ra);
                break;
            }
            case TW_OP_LINK: wr = true; wv = (int64_t)cp(dv->out_off)[th.w1] + imm; break;
            case TW_OP_RLINK:
                if ((uint64_t)rb >= dv->L) { fail(TW_REP_ERR_INSN); fin = W_STOP; break; }
                wr = true; wv = (int64_t)cp(dv->link_rev)[rb];
                break;
            case TW_OP_SEND: {  // schedule (after d) (deliver ..) unless the link drops it
                uint64_t link = (uint64_t)ra;
                const bool fz = (b & (TW_SEND_VIA_LINK | TW_SEND_VIA_RLINK)) != 0;
                if (b & TW_SEND_VIA_LINK) {  // fused LINK a, imm
                    link = (uint64_t)((int64_t)cp(dv->out_off)[th.w1] + imm);
                } else if (b & TW_SEND_VIA_RLINK) {  // fused RLINK a, r
                    const uint64_t rin = (uint64_t)th.reg((b >> 12) & 3u);
                    if (rin >= dv->L) { fail(TW_REP_ERR_INSN); fin = W_STOP; break; }
                    link = cp(dv->link_rev)[rin];
                }
                if (fz) { wr = true; wv = (int64_t)link; npc = pc + 2; }
                if (link >= dv->L) { fail(TW_REP_ERR_INSN); fin = W_STOP; break; }
                const uint32_t kind = b & 0xFFu;
                const uint32_t pr = (b >> 8) & 3u;
                const int64_t payload = (fz && pr == a) ? (int64_t)link : th.reg(pr);
                uint32_t GAS* op_ = gp(dv->link_ord) + ix(link);
                const uint32_t ord = rfl(*op_);
                st32(op_, ord + 1);
                const uint32_t e = dv->link_table ? rfl(gp(dv->link_table)[ix((size_t)link * dv->D + ord % dv->D)]) : 0u;
                if (e & TW_LINK_DROP) {
                    cw->dr = rfl(cw->dr) + 1;
                    hash_add(th.w1, term(now, TW_KIND_DROP | kind, payload));
                } else {
                    cpc = TW_PC_DELIVER_STUB; cnode = th.w1; cra = 4;
                    q0 = payload; q1 = (int64_t)link; q2 = (int64_t)(e & 0x7FFFFFFFu) + tx_us_w(dv, link, kind);
                    q3 = (int64_t)kind;
                    fin = W_SPAWN;
                }
                break;
            }
            case TW_OP_DELIVER: {  // listener dispatch, ForkStrategy fork_ (MonadDialog.hs:232-256,317)
                const uint64_t link = (uint64_t)th.r1;
                const uint32_t kind = (uint32_t)th.r3;
                const uint32_t dst = cp(dv->link_dst)[link];
                const uint32_t set0 = rfl(gp(dv->bind)[ix(dst)]);
                const uint32_t own = rfl(gp(dv->bind_own)[ix(dst)]), rel = rfl(gp(dv->bind_rel)[ix(dst)]);
                const uint32_t set = own == rel ? 0u : set0;  // owner died: released
                uint32_t lpc = TW_PC_NONE;
                if (set && kind < dv->n_kinds) lpc = cp(dv->lpc)[(size_t)(set - 1) * dv->n_kinds + kind];
                const int64_t p0 = th.r0;
                if (lpc == TW_PC_NONE) {
                    cw->ud = rfl(cw->ud) + 1;
                    hash_add(dst, term(now, TW_KIND_UNDELIV | kind, p0));
                } else if (lpc & TW_LPC_INLINE) {  // ForkStrategy `const id` (MonadDialog.hs:114-117)
                    cw->dl = rfl(cw->dl) + 1;
                    hash_add(dst, term(now, TW_KIND_RECV | kind, p0));
                    hash_flush();
                    th.r0 = p0; th.r1 = (int64_t)link; th.r2 = (int64_t)th.w1; th.r3 = (int64_t)kind;
                    hnode = dst;
                    th.w1 = dst;
                    npc = lpc & ~TW_LPC_INLINE;
                } else {
                    cw->dl = rfl(cw->dl) + 1;
                    hash_add(dst, term(now, TW_KIND_RECV | kind, p0));
                    cpc = lpc; cnode = dst; cra = 4;
                    q0 = p0; q1 = (int64_t)link; q2 = (int64_t)th.w1; q3 = (int64_t)kind;
                    fin = W_SPAWN;
                }
                break;
            }
            case TW_OP_LISTEN:
                if ((uint32_t)imm >= dv->n_sets) { fail(TW_REP_ERR_INSN); fin = W_STOP; break; }
                st32(gp(dv->bind) + ix(th.w1), (uint32_t)imm + 1);
                st32(gp(dv->bind_own) + ix(th.w1), b ? th.w2 : 0xFFFFFFFFu);
                if (b) th.w0 |= F_OWNS << FL_SHIFT;
                break;
            case TW_OP_UNLISTEN:
                st32(gp(dv->bind) + ix(th.w1), 0);
                st32(gp(dv->bind_own) + ix(th.w1), 0xFFFFFFFFu);
                break;
            case TW_OP_TRACE:
                hacc += term(now, TW_KIND_TRACE | ((uint32_t)imm & 0xFFFFu), ra);
                if (dv->trace_cap) trace_rec(th.w1, imm, ra);
                if (b & TW_TRACE_PAIR) {  // fused second TRACE
                    const uint32_t t2 = b & 0x1FFFu;
                    const int64_t r2 = th.reg((b >> 13) & 3u);
                    hacc += term(now, TW_KIND_TRACE | t2, r2);
                    if (dv->trace_cap) trace_rec(th.w1, (int32_t)t2, r2);
                    npc = pc + 2;
                }
                break;
            case TW_OP_TMO_BEGIN: {  // schedule (after t) watchdog (TimedT.hs:373-375)
                const uint32_t tmo = rfl(cw->tmo);
                if (tmo >= dv->T) { fail(TW_REP_ERR_INSN); fin = W_STOP; break; }
                st8(gp(dv->tmo_done) + ix(tmo), 0);
                th.set_reg(a, tmo);
                cpc = TW_PC_WATCHDOG_STUB; cnode = th.w1; cra = 4;
                q0 = (int64_t)(((uint64_t)th.w2 << 32) | slot); q1 = (int64_t)tmo; q2 = KP[imm]; q3 = 0;
                cw->tmo = tmo + 1;
                fin = W_SPAWN;
                break;
            }
            case TW_OP_TMO_END: {
                const uint32_t nf = u_nfr(th);
                const uint32_t fr = nf ? frame(th, slot, nf - 1) : 0u;
                if (nf == 0 || (fr >> 16) != 0) { fail(TW_REP_ERR_INSN); fin = W_STOP; break; }
                u_set_nfr(th, nf - 1);
                if ((fr & 0xFFFFu) < dv->T) st8(gp(dv->tmo_done) + ix(fr & 0xFFFFu), 1);
                break;
            }
            case TW_OP_TMO_FIRE: {
                const uint64_t e = (uint64_t)th.r1;
                thr = e < dv->T && !rfl(gp(dv->tmo_done)[ix(e < dv->T ? e : 0)]);
                tref = th.r0; tcode = TW_EXC_TIMEOUT; tval = 0;
                break;
            }
            default:
                fail(TW_REP_ERR_INSN);
                fin = W_STOP;
                break;
            }
            // an ALU op fused with the NSTORE of its result (TW_ALU_NSTORE)
            if ((b & TW_ALU_NSTORE) && (op == TW_OP_SETI || op == TW_OP_SETK || op == TW_OP_ADDI ||
                                        op == TW_OP_MULI || op == TW_OP_NOW || op == TW_OP_NODE)) {
                st_i64(gp(dv->nvars) + ix((size_t)th.w1 * 4 + (b & 3u)), wv);
                npc = pc + 2;
            }
            if (wr) th.set_reg(a, wv);
            if (thr) throw_to(th, slot, tref, tcode, tval);
            if (fin != W_NONE) {
                if (fin != W_DIED && fin != W_STOP) pc = npc;
                break;
            }
            pc = npc;
            if (status != TW_REP_RUNNING) { fin = W_STOP; break; }
            if (pc >= dv->n_insns) { fail(TW_REP_ERR_INSN); fin = W_STOP; break; }
        }
        if (fin != W_DIED) u_set_pc(th, pc);
        // terminal actions: fork's child is queued at now, then the parent waits 1 µs
        if (fin == W_SPAWN) {
            int64_t ref = 0;
            if (!spawn(cpc, cnode, q0, q1, q2, q3, ref)) {
                fin = W_STOP;
            } else {
                if (cra < 4) th.set_reg(cra, ref);
                yt = now + 1;
                fin = W_YIELD;
            }
        }
        if (fin == W_YIELD) {
            enqueue(th, slot, yt);
            urec_store(hrec(slot), dv->RQ, th, 0, 4);
        } else if (fin == W_EXIT) {
            die(th, slot);
            urec_store(hrec(slot), dv->RQ, th, 0, 1);
        } else if (fin == W_STOP) {
            urec_store(hrec(slot), dv->RQ, th, 0, 4);
        }
    }
};

template <int K>
__global__ void __launch_bounds__(64) tw_wave_kernel(const Dev* dptr, int64_t t_end, uint64_t max_events,
                                                      uint32_t budget) {
    const Dev CAS* dv = cp(dptr);
    const uint32_t r = blockIdx.x;
    if (r >= dv->R) return;
    const uint64_t* sc = gp(dv->scal) + r;
    const size_t R = dv->R;
    const uint32_t status0 = (uint32_t)rfl64(sc[SC_STATUS * R]);
    if (status0 != TW_REP_RUNNING) return;
    Wave<K> W(dv, r);
    W.status = status0;
    W.now = rfl64s((int64_t)sc[SC_NOW * R]);
    W.final_t = rfl64s((int64_t)sc[SC_FINAL_T * R]);
    W.seq = rfl((uint32_t)sc[SC_SEQ * R]);
    W.tidc = rfl((uint32_t)sc[SC_TIDC * R]);
    W.live = rfl((uint32_t)sc[SC_LIVE * R]);
    const uint32_t near_n0 = rfl((uint32_t)sc[SC_NEAR_N * R]);
    W.far_n = rfl((uint32_t)sc[SC_FAR_N * R]);
    W.free_n = rfl((uint32_t)sc[SC_FREE_N * R]);
    W.ftop = rfl((uint32_t)sc[SC_FTOP * R]);
    W.bump = rfl((uint32_t)sc[SC_BUMP * R]);
    __shared__ WCold cold;
    W.cw = (WCold LAS*)&cold;
    __shared__ PQCold pqc;
    W.pc = (PQCold LAS*)&pqc;
    W.pqm = dv->tie_mode == TW_TIE_PQUEUE;
    if (W.pqm) {
        const uint32_t GAS* h = gp(dv->pq_hdr) + (size_t)r * PQ_WORDS;
        pqc.n = rfl(h[PQ_N]); pqc.nfree = rfl(h[PQ_NFREE]); pqc.bump = rfl(h[PQ_BUMP]); pqc.flen = rfl(h[PQ_FLEN]);
        pqc.min = make_uint4(rfl(h[PQ_MIN]), rfl(h[PQ_MIN + 1]), rfl(h[PQ_MIN + 2]), rfl(h[PQ_MIN + 3]));
#pragma unroll
        for (int k = 0; k < 32; ++k) pqc.forest[k] = rfl(h[PQ_FOREST + k]);
    }
    cold.main_exc = rfl((uint32_t)sc[SC_MAIN_EXC * R]);
    cold.tmo = rfl((uint32_t)sc[SC_TMO_CTR * R]);
    cold.trn = rfl((uint32_t)sc[SC_TRACE_N * R]);
    cold.dl = cold.dr = cold.ud = cold.d_th = 0;
    uint32_t pending_main = rfl((uint32_t)sc[SC_PENDING_MAIN * R]);
    const uint64_t events0 = rfl64(sc[SC_EVENTS * R]);
    const uint64_t ev_room64 = max_events > events0 ? max_events - events0 : 0;
    const uint32_t ev_room = ev_room64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)ev_room64;
    W.d_ev = 0;
    W.hacc = 0;
    W.hnode = 0xFFFFFFFFu;
    // far runs: bookkeeping from the scalar block, heads/tails from HBM
#pragma unroll
    for (int j = 0; j < TW_RUNS; ++j) {
        const uint32_t ri = rfl((uint32_t)sc[(SC_RH0 + j) * R]), rn = rfl((uint32_t)sc[(SC_RC0 + j) * R]);
        cold.ri[j] = ri;
        cold.rn[j] = rn;
        uint4 h = make_uint4(0, 0, 0, 0), u = h;
        if (rn) {
            h = *W.runp(j, ri);
            uint32_t tp = ri + rn - 1;
            if (tp >= dv->Cr) tp -= dv->Cr;
            u = *W.runp(j, tp);
        }
        cold.rh_t[j] = (int64_t)(((uint64_t)rfl(h.y) << 32) | rfl(h.x));
        cold.rh_sl[j] = rfl(h.z);
        cold.rh_s[j] = rfl(h.w);
        cold.rt_t[j] = (int64_t)(((uint64_t)rfl(u.y) << 32) | rfl(u.x));
        cold.rt_s[j] = rfl(u.w);
    }
    cold.fh_t = 0; cold.fh_s = cold.fh_sl = 0;
    if (W.far_n) W.set_fh(W.far_ld(0));
    W.far_min();
    // near queue: reloaded from the spill area (per replica, lane layout kept)
    W.nbase = W.now;
    W.near_init();
    const uint32_t NSP = 64u * K;
    if (near_n0) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const uint4 e = gp(dv->near_spill)[(size_t)r * NSP + (size_t)j * 64 + W.lane];
            const bool f = e.z != 0xFFFFFFFFu;
            W.nk[j] = f ? ((uint64_t)(ent_t(e) - W.nbase) << 32) | e.w : ~0ull;
            W.ns[j] = f ? e.z : 0u;
            W.lcnt += f ? 1u : 0u;
        }
        W.lane_rescan();
        W.near_n = near_n0;
        W.gmin = wave_min64(W.lmk);
    }

    bool alive = true;
    for (uint32_t it = 0; it < budget && alive; ++it) {
        URec th;
        uint32_t slot = 0;
        bool run = false;
        if (pending_main) {  // runInSandbox main (TimedT.hs:237): runs at t=0, not a pop
            pending_main = 0;
            urec_load(W.hrec(0), dv->RQ, th);
            W.hnode = th.w1;
            run = true;
        } else {
            if (W.live == 0) { W.status = TW_REP_DONE; break; }  // whileM_ notDone
            if (W.d_ev >= ev_room) break;                        // this call's event cap
            if (W.pqm) {  // PQ.minView (TimedT.hs:242)
                if (rfl(pqc.n) == 0) break;
                const uint4 m = W.pq_min();
                const int64_t t = ent_t(m);
                if (t > t_end) break;  // parked beyond t_end
                W.pq_pop();
                if (W.status != TW_REP_RUNNING) break;
                slot = m.z;
                urec_load(W.hrec(slot), dv->RQ, th);
                // (no superseded entries: a throwTo re-stamps the event in place)
                th.w3 = 0;
                --W.live;
                W.now = t;
                W.hnode = th.w1;
                W.final_t = t;
                ++W.d_ev;
                const uint32_t exc = u_exc(th);
                if (exc) {
                    const int64_t val = (int64_t)(((uint64_t)th.xh << 32) | th.xl);
                    u_set_exc(th, 0);
                    th.xl = th.xh = 0;
                    W.hacc += term0(t, TW_KIND_EXC | exc);
                    if (!(u_flags(th) & (F_STARTED | F_MAIN))) {
                        W.status = TW_REP_ABORTED;
                        cold.main_exc = exc;
                        urec_store(W.hrec(slot), dv->RQ, th, 0, 4);
                    } else {
                        run = W.unwind(th, slot, exc, val);
                    }
                } else {
                    W.hacc += term0(t, TW_KIND_RESUME | u_pc(th));
                    run = true;
                }
                if (run) W.step(th, slot);
                W.hash_flush();
                alive = W.status == TW_REP_RUNNING;
                continue;
            }
            // PQ.minView: the near minimum or the far minimum
            if (W.far_dirty) W.far_min();
            const int src = W.fm_src;
            const int64_t ft = W.fm_t;
            const uint32_t fs = W.fm_s, fsl = W.fm_sl;
            const bool use_near = W.near_n != 0;
            const int64_t tn = W.nbase + (int64_t)(W.gmin >> 32);
            const bool use_far = src >= 0 && (!use_near || tless(ft, fs, tn, (uint32_t)W.gmin));
            if (!use_near && !use_far) break;
            const int64_t t = use_far ? ft : tn;
            const uint32_t sq = use_far ? fs : (uint32_t)W.gmin;
            if (t > t_end) break;  // parked beyond t_end
            if (use_far) {
                slot = fsl;
                if (src == TW_RUNS) W.heap_pop();
                else W.run_pop(src);
            } else {
                slot = W.near_pop();
                if (W.status != TW_REP_RUNNING) break;
            }
            urec_load(W.hrec(slot), dv->RQ, th);
            if (th.w3 != sq) continue;  // superseded by a throwTo re-stamp
            th.w3 = 0;
            --W.live;
            W.now = t;                  // curTime .= timestamp (TimedT.hs:241-247)
            if (t - W.nbase > (int64_t)0x7FFFFFFF) W.near_rebase(t);
            W.hnode = th.w1;
            W.final_t = t;
            ++W.d_ev;
            const uint32_t exc = u_exc(th);  // asyncExceptions . at tid <<.= Nothing (:252)
            if (exc) {
                const int64_t val = (int64_t)(((uint64_t)th.xh << 32) | th.xl);
                u_set_exc(th, 0);
                th.xl = th.xh = 0;
                W.hacc += term0(t, TW_KIND_EXC | exc);
                if (!(u_flags(th) & (F_STARTED | F_MAIN))) {  // escapes launchTimedT (:252-263)
                    W.status = TW_REP_ABORTED;
                    cold.main_exc = exc;
                    urec_store(W.hrec(slot), dv->RQ, th, 0, 4);
                } else {
                    run = W.unwind(th, slot, exc, val);
                }
            } else {
                W.hacc += term0(t, TW_KIND_RESUME | u_pc(th));
                run = true;
            }
        }
        if (run) W.step(th, slot);
        W.hash_flush();
        alive = W.status == TW_REP_RUNNING;
    }
    W.hash_flush();
    if (W.status == TW_REP_RUNNING && W.live == 0 && !pending_main) W.status = TW_REP_DONE;

    uint64_t* so = gp(dv->scal) + r;
    if (W.lane == 0) {
        so[SC_PENDING_MAIN * R] = pending_main;
        so[SC_NOW * R] = (uint64_t)W.now; so[SC_FINAL_T * R] = (uint64_t)W.final_t;
        so[SC_SEQ * R] = W.seq; so[SC_TIDC * R] = W.tidc; so[SC_LIVE * R] = W.live;
        so[SC_NEAR_N * R] = W.near_n; so[SC_FAR_N * R] = W.far_n;
        so[SC_STATUS * R] = W.status; so[SC_MAIN_EXC * R] = cold.main_exc;
        so[SC_FREE_N * R] = W.free_n; so[SC_FTOP * R] = W.ftop; so[SC_BUMP * R] = W.bump;
        so[SC_TMO_CTR * R] = cold.tmo; so[SC_TRACE_N * R] = cold.trn;
        so[SC_EVENTS * R] = events0 + W.d_ev;
        so[SC_DELIVERED * R] += cold.dl; so[SC_DROPPED * R] += cold.dr;
        so[SC_UNDELIV * R] += cold.ud; so[SC_THREADS * R] += cold.d_th;
#pragma unroll
        for (int j = 0; j < TW_RUNS; ++j) {
            so[(SC_RH0 + j) * R] = cold.ri[j];
            so[(SC_RC0 + j) * R] = cold.rn[j];
        }
    }
    // spill the near queue verbatim: entry j of lane l at [r][j * 64 + l]
    // (absolute times; an empty entry is written as slot 0xFFFFFFFF)
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const bool f = W.nk[j] == ~0ull;
        gp(dv->near_spill)[(size_t)r * NSP + (size_t)j * 64 + W.lane] =
            f ? make_uint4(0, 0, 0xFFFFFFFFu, 0) : ent(W.nbase + (int64_t)(W.nk[j] >> 32), W.ns[j], (uint32_t)W.nk[j]);
    }
    bool active = W.status == TW_REP_RUNNING && W.d_ev < ev_room;
    int64_t tn = INT64_MAX;
    if (W.pqm) {
        if (rfl(pqc.n)) tn = ent_t(W.pq_min());
        if (W.lane == 0) {
            uint32_t* h = gp(dv->pq_hdr) + (size_t)r * PQ_WORDS;
            h[PQ_N] = pqc.n; h[PQ_NFREE] = pqc.nfree; h[PQ_BUMP] = pqc.bump; h[PQ_FLEN] = pqc.flen;
            h[PQ_MIN] = pqc.min.x; h[PQ_MIN + 1] = pqc.min.y; h[PQ_MIN + 2] = pqc.min.z; h[PQ_MIN + 3] = pqc.min.w;
            for (int k = 0; k < 32; ++k) h[PQ_FOREST + k] = pqc.forest[k];
        }
    } else {
        if (W.near_n) tn = W.nbase + (int64_t)(W.gmin >> 32);
        W.far_min();
        if (W.fm_src >= 0 && W.fm_t < tn) tn = W.fm_t;
    }
    if (active && (tn == INT64_MAX || tn > t_end) && !pending_main) active = false;
    if (active && W.lane == 0)
        __hip_atomic_fetch_add(gp(dv->n_active), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

// near-queue entries per lane (K): 32 for few replicas (<= 4096: C5's
// hotspot receiver keeps 1-2k events on chip), else 4; TW_WAVE_K=4|24|32
// overrides (tests run the tie-audit and random-program cases under each)
int wave_near_k(uint32_t R) {
    if (const char* k = getenv("TW_WAVE_K")) {
        const int v = atoi(k);
        if (v == 4 || v == 24 || v == 32) return v;
    }
    return R <= 4096 ? 32 : 4;
}
size_t wave_spill_entries(uint32_t K) { return 64u * (size_t)K; }

// Host launcher (engine.hip's tw_run): one 64-lane workgroup per replica;
// K is the one tw_load chose (Dev::wave_k: the spill area is sized for it).
hipError_t wave_launch(const Dev& d, const Dev* d_dev, hipStream_t st, int64_t t_end, uint64_t limit,
                       uint32_t budget) {
    // the kernel reads the context from device memory (scalar loads on use),
    // not from kernel arguments held in scalar registers for the whole launch
    hipError_t e = hipMemcpyAsync((void*)d_dev, &d, sizeof(Dev), hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return e;
    if (d.wave_k == 32)
        hipLaunchKernelGGL((tw_wave_kernel<32>), dim3(d.R), dim3(64), 0, st, d_dev, t_end, limit, budget);
    else if (d.wave_k == 24)
        hipLaunchKernelGGL((tw_wave_kernel<24>), dim3(d.R), dim3(64), 0, st, d_dev, t_end, limit, budget);
    else if (d.wave_k == 4)
        hipLaunchKernelGGL((tw_wave_kernel<4>), dim3(d.R), dim3(64), 0, st, d_dev, t_end, limit, budget);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace tw
