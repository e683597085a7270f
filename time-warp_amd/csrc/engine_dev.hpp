// engine_dev.hpp — the device code of libtimewarp.so's event engine (engine.hip):
// the lane-per-replica / logical-process event loop (Lane, tw_run_kernel) and
// the window-loop kernels.  Included by engine.hip.
#pragma once
#include "tw_dev.hpp"

#define TW_NEAR_CAP 16          // on-chip queue entries per replica (LDS)
#define TW_WG 256               // lanes per workgroup (4 waves share one program image)
// Sparse geometry (few replicas: at most a few per SIMD): 16 replicas per
// workgroup, one workgroup per CU, so each replica gets ~10 KB of LDS and a
// 768-entry near heap (most of a hotspot receiver's backlog stays on chip).
#define TW_WG_SPARSE 16
#define TW_NEAR_SPARSE 768
// (One 16-lane wave: spreading them as 4 waves of 4 lanes over the CU's four
// SIMDs measured the same C5 rate, 0.240 vs 0.245 G events/s -- a hotspot
// replica's events are a chain of dependent HBM round trips, not issue.)
// Half geometry (replica-dense runs): the dense LDS layout (256 replicas per
// workgroup) served by 8 waves of 32 active lanes, so 64k replicas fill two
// waves per SIMD; that instance is built for 256 registers so both fit, and
// one wave's scalar, LDS and branch issue overlaps the other's VALU and
// memory waits.
#define TW_HALF_LANES 32
// LP mode (node-partitioned C4): 128 nodes per workgroup and no far-run LDS
// (LP nodes queue few events), so three workgroups share a CU's LDS
#define TW_WG_LP 128
#define TW_NEAR_LP 8      // an LP node queues few events: 8 on chip (4 workgroups per CU)
#define TW_NEAR_COMPACT 8 // compact geometry: 8 on-chip entries per replica, no far runs
// work-list buckets by pending delivery records (tw_lp_compact).  Measured
// with 4 buckets: C4 1.45 vs 1.58 G events/s -- pending records do not predict
// a node's events in the window (most arrive for later windows) -- so 1.
// LP event kernel: a context of more lanes than this many workgroups hold
// (16384 x 128 = 2M) launches this many, walking the work list grid-stride
#define TW_LP_GRID 16384u
#ifndef TW_LP_NB
#define TW_LP_NB 1
#endif
// narrow geometry (fewer replicas than fill the GPU, e.g. C3 sharded 8 ways =
// 8192 per GPU): the dense layout and near heap with TW_NARROW replicas per
// workgroup and one wave per workgroup, so the waves spread over all CUs.
// C3 at 8192 replicas, G events/s by lanes per wave: 8: 1.47, 16: 1.88,
// 32: 2.19, 64: 2.51 (dense, 4 waves per workgroup: 2.35)
#ifndef TW_NARROW
#define TW_NARROW 64
#endif
#define TW_STEP_CAP (1u << 22)  // instructions per thread step (== oracle kStepCap)
// store only the record quads an event changed (1), or the whole record of a
// thread that stays queued (0, the default).  C3, quad-major records, r02:
// 1 = 72 B written per event at 17.2 G events/s, 0 = 90 B at 17.8 G (the
// register compares cost more issue than the bytes save: not HBM-bound)
#ifndef TW_DIRTY_TAIL
#define TW_DIRTY_TAIL 0
#endif
// store-tail sinks: 8 XCD groups x 4 quads x 256 lanes (record quads), then
// one 16-B word per replica (the hash atomic's, kept apart: atomics to shared
// addresses would serialise)
#define TW_DUMMY_Q (8u * 256u)
#define TW_DUMMY_REC (4u * TW_DUMMY_Q)
// cold words (CW_*) in registers (1) or in the LDS cold-word array (0, the
// default): in registers the dense kernel needs 68 AGPRs of spill space and
// ran C3 at 16.5 vs 17.9 G events/s (r02)
#ifndef TW_CW_REGS
#define TW_CW_REGS 0
#endif
#define TW_TAIL_VMEM 9          // vector-memory ops of every iteration after the record prefetch

// LP event kernel: waves per SIMD it is built for (2: <= 256 registers, which
// spills; 1: the AGPRs too, no scratch)
// LP lanes: the per-lane interpreter pass (PL: a hot pass serves lanes at
// different pcs) -- 0 for the A/B of the opcode-uniform pass
#ifndef TW_LP_PL
#define TW_LP_PL 0
#endif
// the record prefetch as the compiler's LDS-DMA builtin (1) or inline asm (0)
#ifndef TW_DMA_BUILTIN
#define TW_DMA_BUILTIN 0
#endif
#ifndef TW_LP_FOLDJ
#define TW_LP_FOLDJ 1  // the LP kernels fold a jump into the pass before it (Lane::FOLDJ; 0: the A/B baseline)
#endif
// the run geometries' lock-step fast path (Lane::fast_run): measured slower
// (C3 138.8 -> 144.3 ms per step), so off -- 1 builds it for A/B
#ifndef TW_FAST
#define TW_FAST 0
#endif
#ifndef TW_FAST_COMPACT
#define TW_FAST_COMPACT 0  // ... in the compact geometry (C2)
#endif
#define TW_FAST_MAX 32u  // instructions per fast_run entry
#ifndef TW_LP_FORKN
#define TW_LP_FORKN 1  // the LP kernels run a counted cross-node fork loop in one pass (Lane::fork_loop; 0: A/B)
#endif
#ifndef TW_LP_WAVES
#define TW_LP_WAVES 2
#endif
#define P_COUNT 36
#define TW_BPROF 8  // diagnostic build: tw_lp_batch's phase cycles after the two P_COUNT sets
// Diagnostic build (-DTW_STATS, lib/libtimewarp_stats.so): per-lane event-path
// counters summed into Dev::prof at kernel end (tools/stats_probe.py).  The
// product build compiles every STAT to nothing.
#ifdef TW_STATS
#define STAT(i) (++st[(i)])
#define STATL(i) (++L.st[(i)])
#else
#define STAT(i) ((void)0)
#define STATL(i) ((void)0)
#endif
enum { K_POP, K_SUPERSEDED, K_PEEK_PF, K_PEEK_HBM, K_PUT_HBM, K_PUT_DEAD, K_PF_ISSUE, K_HASH_IMM, K_HASH_FLUSH,
       K_NEAR_PUSH, K_RUN_PUSH, K_FAR_PUSH, K_INSN, K_CYC_POP, K_CYC_INTERP, K_CYC_TAIL,
       K_CYC_SEL, K_CYC_FETCH, K_CYC_QPOP, K_CYC_COMMIT, K_CYC_PF, K_CYC_TERM, K_CYC_STORE, K_CYC_HASH,
       K_CYC_SPAWN, K_CYC_ENQ, K_SPAWN, K_ALLOC_LD, K_ITER, K_CYC_SEND, K_CYC_DELIV, K_CYC_DUE, K_CYC_PRO,
       K_CYC_EPI, K_CYC_IP, K_PASS };
#ifdef TW_STATS
#define STIME(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define STADD(i, v) (st[(i)] += (uint32_t)(v))
#define STADDL(i, v) (L.st[(i)] += (uint32_t)(v))
#else
#define STIME(v) ((void)0)
#define STADD(i, v) ((void)0)
#define STADDL(i, v) ((void)0)
#endif

// m0 is set by the LDS-DMA (global_load_lds) inline asm only; no other code of
// these kernels uses it.  Each LDS-DMA load and each hand-counted wait that
// proves one landed carries a `; tw:<stream>` comment (pf: the record
// prefetch, run: a far run's next entry) for tools/waitcnt_audit.py, which
// checks every counted wait against the compiled code's paths.
#pragma clang diagnostic ignored "-Winline-asm"

namespace {

using namespace tw;

// Cold per-lane words in LDS, [CW_*][TW_WG] u32: the far runs' bookkeeping,
// the far-heap top, rarely-touched counters and the step's spawn/yield
// staging.  Keeping them out of registers leaves the event loop a small
// register footprint (one wave per SIMD issues every instruction itself; a
// large live set turns into register shuffles on every path).
// The far runs' bookkeeping, as quads in LDS [RQ_*][TW_WG]: head and second
// entry of each run in the queue-entry format {t lo, t hi, slot, seq}, the
// tail {t lo, t hi, seq, length}, and the four head indices in one quad.
static_assert(TW_RUNS == 4, "run head indices share one quad");
enum { RQ_HEAD = 0, RQ_SEC = TW_RUNS, RQ_TAIL = 2 * TW_RUNS, RQ_IDX = 3 * TW_RUNS, RQ_COUNT };

enum {
    CW_FTL = 0,                     // far heap top (t, seq, slot)
    CW_FTH, CW_FS, CW_FSL,
    CW_DL, CW_DR, CW_UD, CW_MAINEXC, CW_TMO,          // counters
    CW_CSP, CW_CNODE,  // step staging: the child's pc | ref register << 16 | registers' source << 20 (csp_word), its node
    CW_DUMMY,                                          // target of idle lanes' predicated stores
    CW_LP_COUNT,  // (LP lanes keep the words above only: the ones below are the replica kernels')
    CW_F2L = CW_LP_COUNT, CW_F2H, CW_F2S,  // the far sources' runner-up key (t, seq): the least but the chosen source's
    CW_VS,                   // victim headers staged at this pop: d_ev << 3 | n0 << 2 | quads (stage_victims)
    CW_TRN,                                            // TRACE records emitted (tw_set_trace: replica contexts)
    CW_COUNT
};
// cold words per lane: LP lanes have no far runs, victim staging or TRACE
// records, and five words less per lane (2.5 KB per 128-lane workgroup) let
// four LP workgroups share a CU's LDS instead of three
template <bool LP>
__host__ __device__ constexpr int cw_count() { return LP ? CW_LP_COUNT : CW_COUNT; }
// the spawn staging word: the child's pc (16 bits, as a thread record keeps
// it), the parent register its ref goes to (4: none) and where the child's
// registers come from (2: the parent's; 0: Lane::qq; 1: LP's deliverer)
__host__ __device__ constexpr uint32_t csp_word(uint32_t pc, uint32_t ra, uint32_t del) {
    return (pc & 0xFFFFu) | (ra << 16) | (del << 20);
}
// byte offset of the child-register quads (Lane::qq) from the record staging
template <int WG, int NC, bool HR>
__host__ __device__ constexpr uint32_t qq_lds_offset() {
    return (uint32_t)(((HR ? 5 : 4) + (HR ? RQ_COUNT : 0)) * WG * 16 + NC * WG * 8 + 4 * WG * 8);
}

// LP-only cold words, after the CW_* block: the due run of a heavy lane
// (head | count << 16, seq base, head time) and its inbox base index
// DW_BSET/BOWN/BREL: LP -- the lane's own listener binding (bind, bind_own,
// bind_rel), cached at the lane's start: only this lane's threads change it
enum { DW_HN, DW_SQ0, DW_TL, DW_TH, DW_IB, DW_BSET, DW_BOWN, DW_BREL, DW_COUNT };

// Pre-decoded instruction class ("uop" flags, built once per launch in the
// kernel prologue from the program image): the interpreter's hot pass computes
// register results, jumps and yields with a few wave-uniform selects and
// enters the per-opcode switch only for the rare ops (U_FX).
enum : uint32_t {
    A_NONE, A_IMM, A_K, A_ADDI, A_MULI, A_MOV, A_ADD, A_SUB, A_NOW, A_NODE, A_TID,  // r[a] <- ...
};
enum : uint32_t { TK_NONE, TK_WREL, TK_WABS, TK_WREG, TK_EXIT, TK_FORK };          // the step ends with ...
// Jumps are an 8-entry truth table over (r[a]==r[b], r[a]<r[b], r[a]==simm16),
// indexed by those three bits: `pc <- imm` is a shift and a select, no branch.
enum : uint32_t {
    JM_NONE = 0x00, JM_ALWAYS = 0xFF, JM_EQ = 0xAA, JM_NE = 0x55, JM_LT = 0xCC, JM_LE = 0xEE, JM_EQI = 0xF0, JM_NEI = 0x0F
};
#define U_ALU(f) ((f) & 0xFu)
#define U_TK(f) (((f) >> 8) & 7u)
#define U_FX (1u << 12)
#define U_TR (1u << 13)                // TRACE: a hash term of r[a]
#define U_LD(f) (((f) >> 14) & 3u)     // table load into r[a]
#define U_JM(f) (((f) >> 16) & 0xFFu)
enum : uint32_t { LD_NONE, LD_NV, LD_OUT, LD_RL };  // node var / out-link base / reverse link
// fused pairs (timewarp.h TW_ALU_NSTORE / TW_TRACE_PAIR): the pass also stores
// r[a] to node var b & 3 / adds the second TRACE's term, and skips the pair's
// second instruction
#define U_NS (1u << 24)
#define U_TR2 (1u << 25)
#define U_P2 (1u << 26)
// END folded into the pass before it (set in the launch prologue from the
// image): the instruction at pc + 1 / pc + 2 (a fused pair's successor) / its
// jump target is END.  Not part of the opcode-uniform pass's flag match.
#define U_NE (1u << 27)
#define U_NE2 (1u << 28)
#define U_JE (1u << 29)
// ... and a wait (WAIT_REL / WAIT_ABS) or a jump at pc + 1 folded the same
// way: the thread yields from this pass (`catch`/`listen` then
// `sleepForever`), or takes the jump with the registers this pass left (a
// counted loop's `addi ; jlt`, `node ; jnei`)
#define U_NW (1u << 30)
#define U_NJ (1u << 31)
#define U_FOLD (U_NE | U_NE2 | U_JE | U_NW | U_NJ)
// (LP prologue) a counted fork loop's head: FORK onto a register's node, then
// `ADDI x,k ; J* .., pc` back to it (`forM_ [..] $ fork ...`, Lane::fork_loop)
#define U_FL (1u << 4)
__host__ __device__ __forceinline__ constexpr uint32_t uop_of(uint32_t op) {
    auto u = [](uint32_t alu, uint32_t jm, uint32_t tk) { return alu | (tk << 8) | (jm << 16); };
    switch (op) {
    case TW_OP_NOP: return 0;
    case TW_OP_END: return u(A_NONE, JM_NONE, TK_EXIT);
    case TW_OP_WAIT_REL: return u(A_NONE, JM_NONE, TK_WREL);
    case TW_OP_WAIT_ABS: return u(A_NONE, JM_NONE, TK_WABS);
    case TW_OP_WAIT_REG: return u(A_NONE, JM_NONE, TK_WREG);
    case TW_OP_FORK: return u(A_NONE, JM_NONE, TK_FORK);
    case TW_OP_MYTID: return u(A_TID, JM_NONE, TK_NONE);
    case TW_OP_SETI: return u(A_IMM, JM_NONE, TK_NONE);
    case TW_OP_SETK: return u(A_K, JM_NONE, TK_NONE);
    case TW_OP_ADDI: return u(A_ADDI, JM_NONE, TK_NONE);
    case TW_OP_MULI: return u(A_MULI, JM_NONE, TK_NONE);
    case TW_OP_MOV: return u(A_MOV, JM_NONE, TK_NONE);
    case TW_OP_ADD: return u(A_ADD, JM_NONE, TK_NONE);
    case TW_OP_SUB: return u(A_SUB, JM_NONE, TK_NONE);
    case TW_OP_JMP: return u(A_NONE, JM_ALWAYS, TK_NONE);
    case TW_OP_JEQ: return u(A_NONE, JM_EQ, TK_NONE);
    case TW_OP_JNE: return u(A_NONE, JM_NE, TK_NONE);
    case TW_OP_JLT: return u(A_NONE, JM_LT, TK_NONE);
    case TW_OP_JLE: return u(A_NONE, JM_LE, TK_NONE);
    case TW_OP_JEQI: return u(A_NONE, JM_EQI, TK_NONE);
    case TW_OP_JNEI: return u(A_NONE, JM_NEI, TK_NONE);
    case TW_OP_NOW: return u(A_NOW, JM_NONE, TK_NONE);
    case TW_OP_NODE: return u(A_NODE, JM_NONE, TK_NONE);
    case TW_OP_TRACE: return U_TR;
    case TW_OP_NLOAD: return LD_NV << 14;
    case TW_OP_LINK: return LD_OUT << 14;
    case TW_OP_RLINK: return LD_RL << 14;
    default: return U_FX;  // every other opcode (and invalid ones) takes the switch
    }
}
__host__ __device__ __forceinline__ constexpr uint32_t uop_insn(uint32_t w0) {
    const uint32_t op = w0 & 0xFFu, b = w0 >> 16;
    uint32_t f = uop_of(op);
    if (b & TW_ALU_NSTORE) {
        if (op == TW_OP_SETI || op == TW_OP_SETK || op == TW_OP_ADDI || op == TW_OP_MULI || op == TW_OP_NOW ||
            op == TW_OP_NODE)
            f |= U_NS | U_P2;
        if (op == TW_OP_TRACE) f |= U_TR2 | U_P2;
    }
    return f;
}

// A load's result consumed in a branch of the interpreter must not stay
// "pending" in the compiler's bookkeeping past that branch: the loop header
// would otherwise wait vmcnt(0) on every pass, i.e. for the record prefetch
// and the previous store tail.  Paths that load already waited for it.
__device__ __forceinline__ void tw_vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// atomic min on a word every lane of a window bounds (the window's record
// minimum, the next event time): a plain read first skips the atomic unless
// it can lower the value, so the L2 does not serialise a million same-address
// atomics per window
__device__ __forceinline__ void min_hot(uint64_t GAS* p, uint64_t v) {
    if (v < __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Claim k consecutive entries of a shared append counter for every lane
// running this code (the active lanes of a divergent region): one atomic per
// wave by its first active lane (ballot-aggregated), each lane's share placed
// by its rank among the active lanes.  Every sender of a hotspot appends to the
// one outbox counter; per-lane atomics on it serialise in the L2.
__device__ __forceinline__ uint32_t wave_append(uint32_t GAS* ctr, uint32_t k) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(true);
    const uint32_t lead = (uint32_t)__builtin_ctzll(m);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    uint32_t base = 0;
    if (below == 0)
        base = __hip_atomic_fetch_add(ctr, k * (uint32_t)__builtin_popcountll(m), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
    base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)lead);
    return base + k * below;
}

__device__ __forceinline__ void lp_deliver(const Dev& c, uint4 a, uint4 b, uint64_t GAS* tmin, int64_t wend,
                                           bool upd_min = true);

// The order delivery records enter a logical process's queue (light drain and
// tw_lp_due alike): (t, link, payload, src, kind), so queue seqs do not depend
// on the order the records arrived in.  a/c: {t lo, t hi, payload lo, payload
// hi}; b/d: {link, kind, src, dst}.
__device__ __forceinline__ bool rec_less(uint4 a, uint4 b, uint4 c, uint4 d) {
    const int64_t t1 = ent_t(a), t2 = ent_t(c);
    if (t1 != t2) return t1 < t2;
    if (b.x != d.x) return b.x < d.x;
    const uint64_t p1 = ((uint64_t)a.w << 32) | a.z, p2 = ((uint64_t)c.w << 32) | c.z;
    if (p1 != p2) return p1 < p2;
    if (b.z != d.z) return b.z < d.z;
    return b.y < d.y;
}

template <bool B>
struct BoolC {
    static constexpr bool value = B;
};

// IP: fork children run in place (fork_in_place) -- the variant the host
// launches under the tie orders where a forked child is always the next pop
template <bool LP, int WG, int NC, bool RUNS = true, bool IP = false>
struct Lane {
    // the replica kernels keep monotone far runs (LDS bookkeeping + HBM FIFOs)
    // unless built without them (the compact geometry: far events go to the
    // HBM heap only, and the LDS a lane needs halves)
    static constexpr bool HR = !LP && RUNS;
    // END folded into the pass before it (U_FOLD): the run geometries only --
    // the compact and LP kernels measured slower with it (C2 -4 %, C5 -2.6 %:
    // their register budget, 254-256 VGPRs at two waves per SIMD)
    static constexpr bool FOLD = HR;
    // the LP kernels fold only a jump (U_NJ): a main thread's counted fork loop
    // (`forM_ [1..N] fork`, examples/token-ring/Main.hs:65-68) takes two passes
    // per fork instead of three
    static constexpr bool FOLDJ = HR || (LP && TW_LP_FOLDJ);
    // the lock-step fast path (fast_run): the run geometries
    static constexpr bool FAST = (HR && TW_FAST) || (!LP && !RUNS && TW_FAST_COMPACT);
    // per-lane hot passes (lanes at different hot ops share a pass) pay off where
    // lanes diverge -- logical processes and the few-replica sparse geometry; the
    // dense replica geometry runs lock-step programs and keeps the cheaper
    // opcode-uniform pass
    static constexpr bool PL = (LP && TW_LP_PL) || WG < 64;
    Dev c;  // by value: kernel arguments stay in SGPRs
    uint32_t r;       // replica
    // LDS (lane-offset pointers; element j at [j * WG])
    uint64_t LAS* nk;     // near heap keys: (t - nbase) << 32 | seq; a free position holds ~0
    uint32_t LAS* ns;     // near heap slots
    int64_t LAS* rf;      // the running thread's registers r0..r3 during its step
    uint4 LAS* pfs;       // prefetch staging: quad q of the next pop's record at [q * WG]
    uint32_t pfs_wave;    // LDS byte address of this wave's staging (quad 0), wave-uniform
    uint32_t LAS* cw;     // cold words [CW_*] in LDS (TW_CW_REGS=0)
    // a spawning instruction's child registers (4 x int64) as two lane-contiguous
    // quads [2][WG]: one 16-B LDS access per pair, and at a pop whose step opens
    // with throwTo the LDS-DMA target of the victims' header quads (stage_victims)
    uint4 LAS* qq;
    // cold words in registers (replica kernels): every index is a constant, so no
    // LDS round trip; the allocator parks them in AGPRs when tight.  The LP
    // kernel runs two waves per SIMD (no AGPR room) and keeps them in LDS.
    static constexpr bool CWR = TW_CW_REGS && !LP;
    uint32_t cwr[CW_COUNT];
    uint4 LAS* rq;        // far runs' bookkeeping quads [RQ_*]
    const uint2 LAS* P;   // program image
    const uint32_t LAS* PU;  // its uop flags
    const uint32_t LAS* PW;  // its pop words (pop_word)
    const int64_t LAS* K; // constant pool
    const uint32_t LAS* LPC;  // listener-set x kind -> handler pc (Dev::lpc), staged in LDS
    // near heap: count, time base, cached root
    uint32_t near_n;
    int64_t nbase;
    uint64_t nrk;  // root key (~0 when empty)
    uint32_t nrs;  // root slot
    // far sources: heap size, and the cached min over the runs and the heap top
    uint32_t far_n;
    bool far_dirty;
    // the running thread's frames / pending-exception quad changed this step
    // (the store tail then writes it; otherwise only the quads that changed)
    bool q1d;
    int fsrc;  // -1 none, 0..TW_RUNS-1 run, TW_RUNS heap
    int64_t fmt;
    uint32_t fms, fmsl;
    // run whose next second entry is in flight into LDS staging quad 4 (-1 none)
    int prun;
    // slot whose record the staging holds or is loading (NONE = invalid)
    uint32_t pf_slot;
    // this iteration's hash terms for the popped thread's node, one atomic at the end
    uint64_t hacc;
    uint32_t hnode;
    // LP: the lane's node's first out-link (LINK never loads it), and the
    // reverse of the link the lane's last delivery came in on (DELIVER loads
    // it with the listener binding, so a handler's reply RLINK never waits)
    uint32_t oo, rlc_link, rlc_rev;
    // free slots: bump pointer + stack with its top in a register
    uint32_t free_n, ftop, bump;
    // replica scalars
    int64_t now, final_t;
    uint32_t seq, tidc, live, status;
    uint32_t d_ev, d_th;  // this launch's event and thread counts
    int64_t t_end;        // this launch's bound (LP: the window's last µs)
    uint32_t ev_room;     // events this launch may still commit
#ifdef TW_STATS
    uint32_t st[P_COUNT];
#endif

    __device__ __forceinline__ size_t ix(size_t i) const { return i * c.R + r; }
    // per-node arrays: replica mode [node][R]; LP mode a lane owns exactly one node
    __device__ __forceinline__ size_t nix(uint32_t node, uint32_t var) const {
        return LP ? ix(var) : ix((size_t)node * 4 + var);
    }
    __device__ __forceinline__ size_t bix(uint32_t node) const { return LP ? ix(0) : ix(node); }
    // LP: the replica this lane's node belongs to (0 for one partitioned
    // scenario), and the global lane of another node of that replica
    __device__ __forceinline__ uint32_t rho() const { return (c.lp0 + r) & ((1u << c.rep_lg) - 1u); }
    __device__ __forceinline__ uint32_t lane_of(uint32_t node) const { return (node << c.rep_lg) | rho(); }
    // link arrays: [link][replica] ([link] x replicas batched, LP)
    __device__ __forceinline__ size_t lix(uint64_t link) const {
        return LP ? ((size_t)link << c.rep_lg) + rho() : ix(link);
    }
    __device__ __forceinline__ size_t tix(uint64_t link, uint32_t ord) const {
        size_t i = (size_t)link * c.D + ord % c.D;
        return LP ? (i << c.rep_lg) + rho() : ix(i);
    }
    // LP cold words (DW_*)
    __device__ __forceinline__ uint32_t dg(int w) const { return cw[(cw_count<LP>() + w) * WG]; }
    __device__ __forceinline__ void ds(int w, uint32_t v) { cw[(cw_count<LP>() + w) * WG] = v; }
    // cold words
    __device__ __forceinline__ uint32_t cg(int w) const {
        if constexpr (CWR) return cwr[w];
        else return cw[w * WG];
    }
    __device__ __forceinline__ void cs(int w, uint32_t v) {
        if constexpr (CWR) cwr[w] = v;
        else cw[w * WG] = v;
    }
    __device__ __forceinline__ int64_t cg64(int wl, int wh) const {
        return (int64_t)(((uint64_t)cg(wh) << 32) | cg(wl));
    }
    __device__ __forceinline__ void cs64(int wl, int wh, int64_t v) {
        cs(wl, (uint32_t)v);
        cs(wh, (uint32_t)((uint64_t)v >> 32));
    }
    __device__ __forceinline__ void cinc(int w) { cs(w, cg(w) + 1); }
    // the child registers (qq): two int64 per quad
    __device__ __forceinline__ static uint4 q2(int64_t a, int64_t b) {
        return make_uint4((uint32_t)a, (uint32_t)((uint64_t)a >> 32), (uint32_t)b, (uint32_t)((uint64_t)b >> 32));
    }
    __device__ __forceinline__ static int64_t qa(uint4 q) { return (int64_t)(((uint64_t)q.y << 32) | q.x); }
    __device__ __forceinline__ static int64_t qb(uint4 q) { return (int64_t)(((uint64_t)q.w << 32) | q.z); }
    __device__ __forceinline__ void qset(int64_t r0, int64_t r1, int64_t r2, int64_t r3) {
        qq[0] = q2(r0, r1);
        qq[WG] = q2(r2, r3);
    }

    __device__ __forceinline__ void fail(uint32_t st) {
        if (status == TW_REP_RUNNING) status = st;
    }
    // The running thread's registers r0..r3: the LDS register file (the
    // interpreter's operand indices are per lane)
    __device__ __forceinline__ int64_t rg(const Th& th, uint32_t i) const { return rf[i * WG]; }
    __device__ __forceinline__ void rs(Th& th, uint32_t i, int64_t v) { rf[i * WG] = v; }

    // ---------------------------------------------------------- near heap (LDS)
    // 4-ary min-heap of unique 64-bit keys; a free position holds ~0, so no
    // read is guarded by the heap size.  NC = 16 (the replica-dense geometry):
    // root + two levels, sift-up and sift-down straight-line code over both
    // levels: the reads of a level are issued together, every move is an
    // unconditional store of a selected value (a "move" onto itself when the
    // entry stays), and no data-dependent branch is taken -- at one wave per
    // SIMD each branch and each dependent LDS round trip costs in full.
    // Larger NC (the sparse geometry, few replicas per CU): sift-up reads the
    // whole ancestor path at once (one round trip), sift-down walks the levels
    // in a wave-uniform loop.
    static constexpr int near_depth() {
        int d = 0;
        long cap = 1, lvl = 1;
        while (cap < NC) { lvl *= 4; cap += lvl; ++d; }
        return d;
    }
    static constexpr int ND = near_depth();  // levels below the root
    static_assert(NC >= 8, "near heap too small");
    __device__ __forceinline__ uint64_t nkey(int64_t t, uint32_t s) const {
        return ((uint64_t)(t - nbase) << 32) | s;
    }
    __device__ __forceinline__ bool near_fits(int64_t t) const {
        return near_n < NC && t - now < c.horizon && (uint64_t)(t - nbase) < 0xFFFFFFFFull;
    }
    __device__ __forceinline__ void near_init() {
#pragma unroll 16
        for (int i = 0; i < NC; ++i) nk[i * WG] = ~0ull;
        near_n = 0;
        nrk = ~0ull; nrs = 0;
    }
    // min of the four children 4p+1..4p+4 of p (positions >= 16 read as ~0)
    __device__ __forceinline__ void near_kids(uint32_t p, uint64_t& kb, uint32_t& sb, uint32_t& ib) const {
        const uint32_t c0 = 4 * p + 1;
        const bool v1 = c0 + 1 < NC, v2 = c0 + 2 < NC, v3 = c0 + 3 < NC;
        const uint32_t a0 = c0 < NC ? c0 : 0, a1 = v1 ? c0 + 1 : 0, a2 = v2 ? c0 + 2 : 0, a3 = v3 ? c0 + 3 : 0;
        uint64_t k0 = nk[a0 * WG], k1 = nk[a1 * WG], k2 = nk[a2 * WG], k3 = nk[a3 * WG];
        const uint32_t s0 = ns[a0 * WG], s1 = ns[a1 * WG], s2 = ns[a2 * WG], s3 = ns[a3 * WG];
        k0 = c0 < NC ? k0 : ~0ull;
        k1 = v1 ? k1 : ~0ull; k2 = v2 ? k2 : ~0ull; k3 = v3 ? k3 : ~0ull;
        const bool m01 = k1 < k0, m23 = k3 < k2;
        const uint64_t ka = m01 ? k1 : k0, kc = m23 ? k3 : k2;
        const uint32_t sa = m01 ? s1 : s0, sc = m23 ? s3 : s2;
        const uint32_t ia = m01 ? c0 + 1 : c0, ic = m23 ? c0 + 3 : c0 + 2;
        const bool m = kc < ka;
        kb = m ? kc : ka; sb = m ? sc : sa; ib = m ? ic : ia;
    }
    // Place (k, s) at the root hole and sift it down.
    __device__ __forceinline__ void near_down(uint64_t k, uint32_t s, bool deep = true) {
        uint64_t k1; uint32_t s1, c1;
        near_kids(0, k1, s1, c1);                // c1 in 1..4
        const bool mv1 = k1 < k;                 // the smallest child rises into the root
        // (the second level holds nothing while every lane's heap has at most
        // five entries: no read of it)
        uint64_t k2 = ~0ull; uint32_t s2 = 0u, c2 = c1;
        if (__builtin_amdgcn_ballot_w64(deep)) near_kids(c1, k2, s2, c2);
        const bool mv2 = mv1 && k2 < k;          // ... and its smallest child into c1
        // root <- c1's entry or k; c1 <- c2's entry, k, or itself; c2 <- k (or
        // c1's new value again when nothing moved that far: a repeated store)
        const uint64_t vb = mv1 ? (mv2 ? k2 : k) : k1;
        const uint32_t sb = mv1 ? (mv2 ? s2 : s) : s1;
        const uint32_t wc = mv2 ? c2 : c1;
        nk[0] = mv1 ? k1 : k;
        ns[0] = mv1 ? s1 : s;
        nk[c1 * WG] = vb;
        ns[c1 * WG] = sb;
        nk[wc * WG] = mv2 ? k : vb;
        ns[wc * WG] = mv2 ? s : sb;
        nrk = mv1 ? k1 : k;
        nrs = mv1 ? s1 : s;
    }
    // Generic NC: place (k, s) at hole p0 and sift it up through the whole
    // ancestor path (read in one round trip; stores top-down so that the
    // clamped repeats of the root are overwritten by the deepest level).
    __device__ __forceinline__ void near_up_from(uint32_t p0, uint64_t k, uint32_t s) {
        uint32_t path[ND + 1];
        uint64_t pk[ND + 2];
        uint32_t ps[ND + 2];
        bool up[ND + 2];
        path[0] = p0;
#pragma unroll
        for (int j = 1; j <= ND; ++j) path[j] = path[j - 1] ? (path[j - 1] - 1) >> 2 : 0u;
#pragma unroll
        for (int j = 1; j <= ND; ++j) { pk[j] = nk[path[j] * WG]; ps[j] = ns[path[j] * WG]; }
        pk[ND + 1] = 0; ps[ND + 1] = 0;
        up[0] = true;
#pragma unroll
        for (int j = 1; j <= ND; ++j) up[j] = up[j - 1] && path[j - 1] != 0 && k < pk[j];
        up[ND + 1] = false;
#pragma unroll
        for (int j = ND; j >= 1; --j) {
            nk[path[j] * WG] = up[j + 1] ? pk[j + 1] : (up[j] ? k : pk[j]);
            ns[path[j] * WG] = up[j + 1] ? ps[j + 1] : (up[j] ? s : ps[j]);
        }
        nk[p0 * WG] = up[1] ? pk[1] : k;
        ns[p0 * WG] = up[1] ? ps[1] : s;
    }
    // Generic NC: place (k, s) at hole p and sift it down (uniform level loop;
    // a lane that stopped rewrites its entry in place).
    __device__ __forceinline__ void near_down_from(uint32_t p, uint64_t k, uint32_t s) {
        bool go = true;
        for (int l = 0; l < ND; ++l) {
            if (!__builtin_amdgcn_ballot_w64(go)) break;
            uint64_t kb; uint32_t sb, ib;
            near_kids(p, kb, sb, ib);
            const bool mv = go && kb < k;
            nk[p * WG] = mv ? kb : k;
            ns[p * WG] = mv ? sb : s;
            go = mv;
            p = mv ? ib : p;
        }
        nk[p * WG] = k;
        ns[p * WG] = s;
    }
    __device__ __forceinline__ void near_push(int64_t t, uint32_t sq, uint32_t slot) {
        if constexpr (NC != 16) {
            STAT(K_NEAR_PUSH);
            const uint64_t k = nkey(t, sq);
            near_up_from(near_n++, k, slot);
            const bool m = k < nrk;
            nrk = m ? k : nrk;
            nrs = m ? slot : nrs;
            return;
        }
        STAT(K_NEAR_PUSH);
        const uint64_t k = nkey(t, sq);
        const uint32_t n = near_n++;
        // parent and grandparent of n (clamped to the root)
        const uint32_t p1 = n ? (n - 1) >> 2 : 0;
        const uint32_t p2 = p1 ? (p1 - 1) >> 2 : 0;
        const uint64_t k1 = nk[p1 * WG], k2 = nk[p2 * WG];
        const uint32_t s1 = ns[p1 * WG], s2 = ns[p2 * WG];
        const bool up1 = n != 0 && k < k1;         // parent moves down into n
        const bool up2 = up1 && p1 != 0 && k < k2;  // grandparent moves down into p1
        // p2 <- k or itself; p1 <- grandparent, k or itself; n <- parent or k.
        // Stored top-down so that when positions coincide (n = 0: all three;
        // n <= 4: p1 = p2 = 0) the last store, the one for the deepest, wins.
        nk[p2 * WG] = up2 ? k : k2;
        ns[p2 * WG] = up2 ? slot : s2;
        nk[p1 * WG] = up2 ? k2 : (up1 ? k : k1);
        ns[p1 * WG] = up2 ? s2 : (up1 ? slot : s1);
        nk[n * WG] = up1 ? k1 : k;
        ns[n * WG] = up1 ? s1 : slot;
        const bool m = k < nrk;
        nrk = m ? k : nrk;
        nrs = m ? slot : nrs;
    }
    __device__ __forceinline__ void near_pop() {
        const uint32_t n = --near_n;
        const uint64_t lk = n ? nk[n * WG] : ~0ull;
        const uint32_t ls = ns[n * WG];
        nk[n * WG] = ~0ull;
        if constexpr (NC != 16) {
            near_down_from(0, lk, ls);
            nrk = nk[0];
            nrs = ns[0];
        } else {
            near_down(lk, ls, n > 5u);
        }
    }
    // Re-key the live near entry with seq `old_seq` (seqs are unique) to (t, sq),
    // an earlier time: remove it (the last entry fills its hole) and push it anew.
    __device__ __forceinline__ bool near_rekey(uint32_t old_seq, int64_t t, uint32_t sq, uint32_t slot) {
        if constexpr (NC != 16) {
            // find the entry, fill its hole with the last entry (sifted whichever
            // way it must go), then push the re-keyed entry
            uint32_t i = 0xFFFFFFFFu;
            for (uint32_t j = 0; j < near_n; ++j) {
                const uint64_t k = nk[j * WG];
                if ((uint32_t)k == old_seq && k != ~0ull) { i = j; break; }
            }
            if (i == 0xFFFFFFFFu) return false;
            const uint32_t n = --near_n;
            const uint64_t lk = nk[n * WG];
            const uint32_t ls = ns[n * WG];
            nk[n * WG] = ~0ull;
            if (i != n) {
                if (i > 0 && lk < nk[((i - 1) >> 2) * WG]) near_up_from(i, lk, ls);
                else near_down_from(i, lk, ls);
            }
            near_up_from(near_n++, nkey(t, sq), slot);
            nrk = nk[0];
            nrs = ns[0];
            return true;
        } else {
        uint32_t hit = 0;
#pragma unroll
        for (int i = 0; i < NC; ++i) {
            const uint64_t k = nk[i * WG];
            hit |= ((uint32_t)k == old_seq && k != ~0ull) ? 1u << i : 0u;
        }
        if (!hit) return false;
        const uint32_t i = (uint32_t)__builtin_ctz(hit);
        // remove i: the last entry fills the hole; it can only need to move down
        // (it was deeper, under a key <= it) or up (below i's ancestors); use a
        // full rebuild of that path by re-pushing all entries above -- rare
        // path (a throwTo of an on-chip thread), so simply rebuild the heap.
        uint64_t kk[NC];
        uint32_t ss[NC];
        const uint32_t n = near_n;
#pragma unroll
        for (int j = 0; j < NC; ++j) { kk[j] = nk[j * WG]; ss[j] = ns[j * WG]; }
        near_init();
        for (uint32_t j = 0; j < n; ++j) {
            if (j == i) continue;
            const uint64_t k = kk[j];
            near_push(nbase + (int64_t)(k >> 32), (uint32_t)k, ss[j]);
        }
        near_push(t, sq, slot);
        return true;
        }
    }
    // Move the near heap to a new time base (keeps (t - nbase) inside 32 bits).
    __device__ __forceinline__ void near_rebase(int64_t nb) {
        const uint64_t d = (uint64_t)(nb - nbase) << 32;
#pragma unroll 16
        for (int i = 0; i < NC; ++i) {
            const uint64_t k = nk[i * WG];
            nk[i * WG] = k == ~0ull ? k : k - d;
        }
        nrk = nrk == ~0ull ? nrk : nrk - d;
        nbase = nb;
    }

    // ------------------------------------------------------ far heap (HBM, 4-ary)
    __device__ __forceinline__ uint4 far_ld(uint32_t i) const { return gp(c.far)[ix(i)]; }
    __device__ __forceinline__ void far_st(uint32_t i, uint4 e) const { gp(c.far)[ix(i)] = e; }
    __device__ __forceinline__ void set_ftop(uint4 e) {
        cs(CW_FTL, e.x); cs(CW_FTH, e.y); cs(CW_FS, e.w); cs(CW_FSL, e.z);
    }
    // Heaps of up to TW_FAR_FAST entries are at most TW_FAR_D levels deep below
    // the root; their sift code reads before it writes: a push reads every
    // ancestor in one batch of independent loads, a pop walks down with loads
    // only, and the moves are stored at the end.  (A load waits for every older
    // store of the wave -- interleaving them would add a store round trip to
    // every level.)  Larger heaps take the plain loops.
#define TW_FAR_D 8
#define TW_FAR_FAST 87380u  // indices below (4^9 - 1) / 3 have at most 8 ancestors
    __device__ __forceinline__ void far_push(int64_t t, uint32_t sq, uint32_t slot) {
        if (far_n >= c.Q) { fail(TW_REP_ERR_QUEUE); return; }
        STAT(K_FAR_PUSH);
        const uint32_t i0 = far_n++;
        const uint4 e = ent(t, slot, sq);
        if (c.Q > TW_FAR_FAST) {
            uint32_t i = i0;
            while (i > 0) {
                uint32_t p = (i - 1) >> 2;
                uint4 q = far_ld(p);
                if (!tless(t, sq, ent_t(q), q.w)) break;
                far_st(i, q);
                i = p;
            }
            far_st(i, e);
            if (i == 0) { set_ftop(e); far_dirty = true; }
            return;
        }
        uint32_t a[TW_FAR_D];
        bool v[TW_FAR_D];
        uint4 q[TW_FAR_D];
        uint32_t cur = i0;
#pragma unroll
        for (int k = 0; k < TW_FAR_D; ++k) {
            v[k] = cur > 0;
            a[k] = v[k] ? (cur - 1) >> 2 : 0u;
            cur = a[k];
        }
#pragma unroll
        for (int k = 0; k < TW_FAR_D; ++k) q[k] = far_ld(a[k]);
        uint32_t hole = i0;
        bool go = true;
#pragma unroll
        for (int k = 0; k < TW_FAR_D; ++k) {
            const bool mv = go && v[k] && tless(t, sq, ent_t(q[k]), q[k].w);
            if (mv) far_st(hole, q[k]);
            hole = mv ? a[k] : hole;
            go = mv;
        }
        far_st(hole, e);
        if (hole == 0) { set_ftop(e); far_dirty = true; }
    }
    __device__ __forceinline__ void far_pop() {
        uint32_t n = --far_n;
        far_dirty = true;
        if (n == 0) return;
        uint4 le = far_ld(n);
        int64_t t = ent_t(le);
        if (c.Q > TW_FAR_FAST) {
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
                if (i == 0) set_ftop(b);
                i = c0 + best;
            }
            far_st(i, le);
            if (i == 0) set_ftop(le);
            return;
        }
        // walk down with loads only; the moves (entry mk[k] into position pk[k]) are stored after
        uint32_t pk[TW_FAR_D];
        uint4 mk[TW_FAR_D];
        bool mvk[TW_FAR_D];
        uint32_t hole = 0;
        bool go = true;
#pragma unroll
        for (int k = 0; k < TW_FAR_D; ++k) {
            const uint32_t c0 = 4 * hole + 1;
            const bool ok = go && c0 < n;
            const uint32_t b0 = ok ? c0 : 0u;
            const uint32_t cn = !ok ? 0u : (n - c0 < 4 ? n - c0 : 4u);
            const uint4 e0 = far_ld(b0);
            const uint4 e1 = far_ld(cn > 1 ? b0 + 1 : b0);
            const uint4 e2 = far_ld(cn > 2 ? b0 + 2 : b0);
            const uint4 e3 = far_ld(cn > 3 ? b0 + 3 : b0);
            uint4 b = e0;
            uint32_t best = 0;
            if (cn > 1 && tless(ent_t(e1), e1.w, ent_t(b), b.w)) { b = e1; best = 1; }
            if (cn > 2 && tless(ent_t(e2), e2.w, ent_t(b), b.w)) { b = e2; best = 2; }
            if (cn > 3 && tless(ent_t(e3), e3.w, ent_t(b), b.w)) { b = e3; best = 3; }
            const bool mv = ok && tless(ent_t(b), b.w, t, le.w);
            pk[k] = hole;
            mk[k] = b;
            mvk[k] = mv;
            hole = mv ? c0 + best : hole;
            go = mv;
        }
#pragma unroll
        for (int k = 0; k < TW_FAR_D; ++k)
            if (mvk[k]) far_st(pk[k], mk[k]);
        far_st(hole, le);
        set_ftop(mvk[0] ? mk[0] : le);
    }

    // ---------------------------------------------------- far runs (HBM FIFOs)
    // Patience-sorting piles: a far event is appended to the run whose tail is
    // the largest key <= it, so runs stay sorted and pops are O(1).  TimedT
    // scenarios park threads in monotone streams (killers at one absolute time,
    // sleepForever timers, re-stamped victims of a killer sweep), so the heap
    // sees only stragglers.  Bookkeeping lives in the cold LDS words; the run
    // indexed by a per-lane number is a per-lane LDS address, not a select chain.
    __device__ __forceinline__ uint4 GAS* run_at(uint32_t j, uint32_t pos) const {
        return gp(c.runs) + ((size_t)j * c.Cr + pos) * c.R + r;
    }
    // the second entry loaded by the last run_pop lands in LDS
    __device__ __forceinline__ uint4 LAS* rqp(int w) const { return rq + w * WG; }
    __device__ __forceinline__ static uint32_t q_at(uint4 q, int j) {
        return j == 0 ? q.x : j == 1 ? q.y : j == 2 ? q.z : q.w;
    }
    // Called after prefetch_all (4 younger vector-memory ops) and before the
    // store tail: vmcnt(4) proves the entry landed without waiting for them.
    __device__ __forceinline__ void run_commit() {
        if constexpr (!HR) return;
        if (prun >= 0) {
            asm volatile("s_waitcnt vmcnt(4) ; tw:run" ::: "memory");
            *rqp(RQ_SEC + prun) = pfs[4 * WG];
            prun = -1;
        }
    }
    __device__ __forceinline__ bool run_push(int64_t t, uint32_t sq, uint32_t slot) {
        if constexpr (!HR) return false;  // LP nodes / the compact geometry: no far runs (no LDS for them either)
        if (c.Cr == 0) return false;
        uint4 tl[TW_RUNS];
#pragma unroll
        for (int j = 0; j < TW_RUNS; ++j) tl[j] = *rqp(RQ_TAIL + j);
        const uint4 ix4 = *rqp(RQ_IDX);
        int best = -1, empty = -1;
        int64_t bt = 0;
        uint32_t bs = 0, bn = 0, brh = 0;
#pragma unroll
        for (int j = 0; j < TW_RUNS; ++j) {
            const uint32_t n = tl[j].w;
            const int64_t ut = (int64_t)(((uint64_t)tl[j].y << 32) | tl[j].x);
            const uint32_t us = tl[j].z;
            const bool e = n == 0 && empty < 0;
            empty = e ? j : empty;
            const bool ok = n != 0 && n < c.Cr && !tless(t, sq, ut, us) && (best < 0 || tless(bt, bs, ut, us));
            best = ok ? j : best;
            bt = ok ? ut : bt;
            bs = ok ? us : bs;
            bn = ok ? n : bn;
            brh = ok ? q_at(ix4, j) : brh;
        }
        if (best < 0 && empty >= 0) { bn = 0; brh = q_at(ix4, empty); }
        const int sel = best >= 0 ? best : empty;
        if (sel < 0) return false;
        STAT(K_RUN_PUSH);
        uint32_t pos = brh + bn;
        if (pos >= c.Cr) pos -= c.Cr;
        const uint4 e = ent(t, slot, sq);
        *run_at(sel, pos) = e;
        if (bn == 0) { *rqp(RQ_HEAD + sel) = e; far_dirty = true; }
        else if (bn == 1) *rqp(RQ_SEC + sel) = e;
        *rqp(RQ_TAIL + sel) = make_uint4(e.x, e.y, sq, bn + 1);
        return true;
    }
    // The head moves to the second entry; the entry after it is loaded now, by
    // LDS-DMA into staging quad 4, and committed before the store tail.
    // The popped run is the far minimum (fsrc); its new head stays the minimum
    // when it is below the runner-up far_min recorded (the least key of the
    // other far sources), so a stream of pops from one run -- C3's teardown: the
    // 4,096 kill wakes at 120 s and the 8,192 victims re-stamped behind them --
    // keeps far_min's eight-quad scan off every pop.
    __device__ __forceinline__ void run_pop(int sel) {
        if constexpr (!HR) return;  // unreachable: fsrc is never a run without runs
        run_commit();
        uint4 ix4 = *rqp(RQ_IDX);
        uint32_t h = q_at(ix4, sel) + 1;
        h = h == c.Cr ? 0 : h;
        ix4.x = sel == 0 ? h : ix4.x; ix4.y = sel == 1 ? h : ix4.y;
        ix4.z = sel == 2 ? h : ix4.z; ix4.w = sel == 3 ? h : ix4.w;
        *rqp(RQ_IDX) = ix4;
        const uint4 nh = *rqp(RQ_SEC + sel);
        *rqp(RQ_HEAD + sel) = nh;
        uint4 tl = *rqp(RQ_TAIL + sel);
        const uint32_t n = --tl.w;
        *rqp(RQ_TAIL + sel) = tl;
        {
            const int64_t t = ent_t(nh);
            const bool keep = !far_dirty && fsrc == sel && n != 0 && tless(t, nh.w, cg64(CW_F2L, CW_F2H), cg(CW_F2S));
            fmt = keep ? t : fmt;
            fms = keep ? nh.w : fms;
            fmsl = keep ? nh.z : fmsl;
            far_dirty = !keep;
        }
        if (n >= 2) {
            const uint32_t p2 = h + 1 == c.Cr ? 0 : h + 1;
            // into LDS staging quad 4 (no register left pending across the step)
            // (readfirstlane: the m0 operand is an SGPR whatever register the value was kept in)
            const uint32_t pw4 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(pfs_wave + 4 * WG * 16));
            asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off ; tw:run" ::"v"(run_at(sel, p2)),
                         "s"(pw4) : "memory", "m0");
            prun = sel;
        }
    }
    __device__ __forceinline__ void far_min() {  // heads only: a pending second entry is not needed
        far_dirty = false;
        fsrc = -1;
        fmt = 0; fms = 0; fmsl = 0;
        if (far_n) { fsrc = TW_RUNS; fmt = cg64(CW_FTL, CW_FTH); fms = cg(CW_FS); fmsl = cg(CW_FSL); }
        if constexpr (LP) {
            // no far runs; the due run of a heavy lane is source 0 (its seqs were
            // reserved at the window's start, in the run's order)
            const uint32_t hn = dg(DW_HN), h = hn & 0xFFFFu;
            if (h < (hn >> 16)) {
                const int64_t t = (int64_t)(((uint64_t)dg(DW_TH) << 32) | dg(DW_TL));
                const uint32_t sq = dg(DW_SQ0) + 1u + h;
                if (fsrc < 0 || tless(t, sq, fmt, fms)) { fsrc = 0; fmt = t; fms = sq; fmsl = 0xFFFFFFFFu; }
            }
            return;
        }
        if constexpr (!HR) return;
        uint4 hd[TW_RUNS], tl[TW_RUNS];
#pragma unroll
        for (int j = 0; j < TW_RUNS; ++j) { hd[j] = *rqp(RQ_HEAD + j); tl[j] = *rqp(RQ_TAIL + j); }
        // (and the runner-up: the least key of the sources but the chosen one;
        // none = (INT64_MAX, ~0), above every key)
        int64_t t2 = INT64_MAX;
        uint32_t s2 = 0xFFFFFFFFu;
#pragma unroll
        for (int j = 0; j < TW_RUNS; ++j) {
            const int64_t t = ent_t(hd[j]);
            const bool v = tl[j].w != 0;
            const bool b = v && (fsrc < 0 || tless(t, hd[j].w, fmt, fms));
            // a new minimum demotes the old one (when there was one); otherwise
            // the head may still be the runner-up
            const bool d = b && fsrc >= 0 && tless(fmt, fms, t2, s2);
            const bool u = v && !b && tless(t, hd[j].w, t2, s2);
            t2 = d ? fmt : (u ? t : t2);
            s2 = d ? fms : (u ? hd[j].w : s2);
            fsrc = b ? j : fsrc;
            fmt = b ? t : fmt;
            fms = b ? hd[j].w : fms;
            fmsl = b ? hd[j].z : fmsl;
        }
        cs64(CW_F2L, CW_F2H, t2);
        cs(CW_F2S, s2);
    }
    // every queued event (near heap, far sources, LP due run) is later than t
    __device__ __forceinline__ bool queue_after(int64_t t) {
        if (far_dirty) far_min();
        const bool nl = near_n == 0 || nbase + (int64_t)(nrk >> 32) > t;
        return nl && (fsrc < 0 || fmt > t);
    }
    __device__ __forceinline__ void push_far(int64_t t, uint32_t sq, uint32_t slot) {
        if (!run_push(t, sq, slot)) far_push(t, sq, slot);
    }

    // ------------------------------------------------------------- queue
    // A fresh insertion counter value, as the key the tie mode gives it.  The
    // counter is 32-bit: reaching its top is a TW_REP_ERR_COUNTER status (the
    // replica stops after this step), never a silent wrap.
    // (TW_TIE_FORKFIRST: 31 bits -- bit 31 of a key marks every entry but a
    // forked child's, `child`, which sorts first among its time's entries)
    __device__ __forceinline__ uint32_t seq_top() const {
        return c.tie_mode == TW_TIE_FORKFIRST ? 0x7FFFFFFFu : 0xFFFFFFFFu;
    }
    __device__ __forceinline__ uint32_t next_seq(bool child = false) {
        if (seq == seq_top()) fail(TW_REP_ERR_COUNTER);
        else ++seq;
        if (child && c.tie_mode == TW_TIE_FORKFIRST) return seq;
        return c.tie_mode ? seq_key(c.tie_mode, seq) : seq;
    }
    // Queue the thread at t with a fresh seq; returns true if the entry is on chip.
    __device__ __forceinline__ bool enqueue(Th& th, uint32_t slot, int64_t t, bool child = false) {
        uint32_t s = next_seq(child);
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

    // ------------------------------------------------- thread records
    // A record lives in HBM while its thread is queued and in registers (the
    // header) + the LDS register file (r0..r3) while it runs.  `pf` holds a
    // prefetched copy of the next pop's record, loaded right after the previous
    // pop so its latency hides behind a whole step.
    __device__ __forceinline__ static void unpack(Th& th, uint4 a, uint4 b, uint4 d, uint4 e) {
        th.w0 = a.x; th.w1 = a.y; th.w2 = a.z; th.w3 = a.w;
        th.f0 = b.x; th.f1 = b.y; th.xl = b.z; th.xh = b.w;
        th.r0 = (int64_t)(((uint64_t)d.y << 32) | d.x);
        th.r1 = (int64_t)(((uint64_t)d.w << 32) | d.z);
        th.r2 = (int64_t)(((uint64_t)e.y << 32) | e.x);
        th.r3 = (int64_t)(((uint64_t)e.w << 32) | e.z);
    }
    // quad 0 of a record; quad q is c.RQ further ([quad][slot][replica]: the 64
    // lanes' same quad of the same slot is one contiguous 1 KiB, so a wave that
    // writes only its header quads still writes whole lines)
    // (LP lanes: a record's four quads contiguous, [slot][lane][quad], c.RQ = 1 --
    // their work lists are sparse, so a record is one line instead of four)
    __device__ __forceinline__ uint4 GAS* hrec(uint32_t slot) const {
        return gp(c.slots) + (LP ? ix(slot) * 4 : ix(slot));
    }
    __device__ __forceinline__ void hbm_load(uint32_t slot, Th& th) const {
        const uint4 GAS* p = hrec(slot);
        unpack(th, p[0], p[c.RQ], p[2 * c.RQ], p[3 * c.RQ]);
    }
    // mode ST_THROUGH: the full record; ST_DEAD: only the header quad (the tid
    // that invalidates stale refs)
    __device__ __forceinline__ void put_hdr(uint32_t slot, const Th& th) {
        if (slot == pf_slot) pf_slot = 0xFFFFFFFFu;
        STAT(K_PUT_DEAD);
        hrec(slot)[0] = make_uint4(th.w0, th.w1, th.w2, th.w3);
    }
    __device__ __forceinline__ void put_rec(uint32_t slot, const Th& th) {
        if (slot == pf_slot) pf_slot = 0xFFFFFFFFu;
        STAT(K_PUT_HBM);
        uint4 GAS* p = hrec(slot);
        p[0] = make_uint4(th.w0, th.w1, th.w2, th.w3);
        p[c.RQ] = make_uint4(th.f0, th.f1, th.xl, th.xh);
        p[2 * c.RQ] = make_uint4((uint32_t)th.r0, (uint32_t)((uint64_t)th.r0 >> 32), (uint32_t)th.r1,
                                 (uint32_t)((uint64_t)th.r1 >> 32));
        p[3 * c.RQ] = make_uint4((uint32_t)th.r2, (uint32_t)((uint64_t)th.r2 >> 32), (uint32_t)th.r3,
                          (uint32_t)((uint64_t)th.r3 >> 32));
    }
    // The iteration's stores: the same NUMBER of vector-memory instructions on
    // every path (so the next pop's counted vmcnt wait proves the prefetch
    // landed without waiting for them), but each lane writes to HBM only what
    // changed: the header quad of its thread (pc, flags, wake seq), the frames /
    // exception quad when q1d, each register quad when its registers differ
    // from the record's, and a forked child's whole record.  A quad with
    // nothing to write goes to the lane's dummy sink (a few L2-resident lines
    // per lane), so no store sits behind a branch or an exec mask.
    __device__ __forceinline__ void store_tail(uint32_t slot, Th& th, bool full, bool hdr, uint32_t cslot,
                                               const Th& ch) {
        // the record sinks are shared by the workgroups of one XCD (blocks are
        // dealt to the 8 XCDs round-robin): a few KiB that stay in that XCD's L2
        // (recomputed here rather than held in registers)
        uint4 GAS* dm = gp(c.dummy) + (size_t)(blockIdx.x & 7u) * 256u + (threadIdx.x & 255u);
        const size_t R5 = TW_DUMMY_Q;
        const int64_t n0 = rg(th, 0), n1 = rg(th, 1), n2 = rg(th, 2), n3 = rg(th, 3);
        const bool w0q = full || hdr;
#if TW_DIRTY_TAIL
        const bool w1q = full && q1d;
        const bool w2q = full && (n0 != th.r0 || n1 != th.r1);
        const bool w3q = full && (n2 != th.r2 || n3 != th.r3);
#else
        const bool w1q = full, w2q = full, w3q = full;
#endif
        th.r0 = n0; th.r1 = n1; th.r2 = n2; th.r3 = n3;
        uint4 GAS* pr = hrec(slot);
        *(w0q ? pr : dm) = make_uint4(th.w0, th.w1, th.w2, th.w3);
        *(w1q ? pr + c.RQ : dm + R5) = make_uint4(th.f0, th.f1, th.xl, th.xh);
        *(w2q ? pr + 2 * c.RQ : dm + 2 * R5) =
            make_uint4((uint32_t)th.r0, (uint32_t)((uint64_t)th.r0 >> 32), (uint32_t)th.r1,
                       (uint32_t)((uint64_t)th.r1 >> 32));
        *(w3q ? pr + 3 * c.RQ : dm + 3 * R5) =
            make_uint4((uint32_t)th.r2, (uint32_t)((uint64_t)th.r2 >> 32), (uint32_t)th.r3,
                       (uint32_t)((uint64_t)th.r3 >> 32));
        const bool hc = cslot != 0xFFFFFFFFu;
        uint4 GAS* pc0 = hrec(hc ? cslot : 0);
        *(hc ? pc0 : dm) = make_uint4(ch.w0, ch.w1, ch.w2, ch.w3);
        *(hc ? pc0 + c.RQ : dm + R5) = make_uint4(ch.f0, ch.f1, ch.xl, ch.xh);
        *(hc ? pc0 + 2 * c.RQ : dm + 2 * R5) =
            make_uint4((uint32_t)ch.r0, (uint32_t)((uint64_t)ch.r0 >> 32), (uint32_t)ch.r1,
                       (uint32_t)((uint64_t)ch.r1 >> 32));
        *(hc ? pc0 + 3 * c.RQ : dm + 3 * R5) =
            make_uint4((uint32_t)ch.r2, (uint32_t)((uint64_t)ch.r2 >> 32), (uint32_t)ch.r3,
                       (uint32_t)((uint64_t)ch.r3 >> 32));
        pf_slot = (w0q && slot == pf_slot) || (hc && cslot == pf_slot) ? 0xFFFFFFFFu : pf_slot;
    }

    // Issue the HBM load of the record the next pop will most likely need,
    // straight into LDS (global_load_lds: no registers held, no compiler-
    // tracked pending load).  Every lane issues it (idle lanes reload slot 0).
    // The iteration then always issues TW_TAIL_VMEM more vector-memory ops (the
    // store tail and the hash atomic), so at the next pop `vmcnt(TW_TAIL_VMEM)`
    // proves the prefetch landed without waiting for those stores.
    __device__ __forceinline__ void prefetch_all(uint32_t cur) {
        if (far_dirty) far_min();
        uint32_t s = 0xFFFFFFFFu;
        if (near_n) s = nrs;
        if (fsrc >= 0 && (!near_n || tless(fmt, fms, nbase + (int64_t)(nrk >> 32), (uint32_t)nrk))) s = fmsl;
        const bool valid = s != 0xFFFFFFFFu && s != cur && s < c.S;
        STAT(K_PF_ISSUE);
        const uint4 GAS* p = hrec(valid ? s : 0u);
#if TW_DMA_BUILTIN
        // the compiler's own LDS-DMA instruction: its vector-memory count is
        // modelled (inline asm is opaque to the wait-count pass, which then
        // guarded the address registers with vmcnt waits where they were reused)
        const uint32_t pw = (uint32_t)__builtin_amdgcn_readfirstlane((int)pfs_wave);
        uint4 LAS* d0 = (uint4 LAS*)(size_t)pw;
        __builtin_amdgcn_global_load_lds((const void GAS*)p, (void LAS*)d0, 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void GAS*)(p + c.RQ), (void LAS*)(d0 + WG), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void GAS*)(p + 2 * c.RQ), (void LAS*)(d0 + 2 * WG), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void GAS*)(p + 3 * c.RQ), (void LAS*)(d0 + 3 * WG), 16, 0, 0);
#else
        // (readfirstlane: the m0 operand is an SGPR whatever register the value was kept in)
        const uint32_t pw = (uint32_t)__builtin_amdgcn_readfirstlane((int)pfs_wave);
        // the instruction offset of global_load_lds also offsets the LDS
        // destination, so each quad gets its own global address instead
        asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off ; tw:pf" ::"v"(p), "s"(pw)
                     : "memory", "m0");
        asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off ; tw:pf" ::"v"(p + c.RQ),
                     "s"(pw + WG * 16) : "memory", "m0");
        asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off ; tw:pf" ::"v"(p + 2 * c.RQ),
                     "s"(pw + 2 * WG * 16) : "memory", "m0");
        asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off ; tw:pf" ::"v"(p + 3 * c.RQ),
                     "s"(pw + 3 * WG * 16) : "memory", "m0");
#endif
        pf_slot = valid ? s : 0xFFFFFFFFu;
    }
    // The popped thread's record: the prefetched copy, or (rarely) a fresh load
    // that the missing lane copies into its own staging quads first.  Every
    // lane then reads the staging quads, so no register stays pending on a
    // load across the merge (which made the compiler wait vmcnt(0) -- for the
    // previous iteration's store tail too -- on the common path).
    __device__ __forceinline__ void fetch_rec(uint32_t slot, Th& th) {
        if (slot != pf_slot) {
            STAT(K_PEEK_HBM);
            const uint4 GAS* p = hrec(slot);
            const uint4 a = p[0], b = p[c.RQ], d = p[2 * c.RQ], e = p[3 * c.RQ];
            pfs[0] = a; pfs[WG] = b; pfs[2 * WG] = d; pfs[3 * WG] = e;
        } else {
            STAT(K_PEEK_PF);
        }
        asm volatile("s_waitcnt vmcnt(%0) ; tw:pf" ::"n"(TW_TAIL_VMEM) : "memory");
        unpack(th, pfs[0], pfs[WG], pfs[2 * WG], pfs[3 * WG]);
    }

    // Free slots: never-used slots come from a bump pointer (no memory read);
    // freed slots form a LIFO stack whose top lives in a register.
    __device__ __forceinline__ uint32_t alloc_slot() {
        if (free_n) {
            uint32_t s = ftop;
            if (--free_n) {
                STAT(K_ALLOC_LD);
                ftop = gp(c.free_stk)[ix(free_n - 1)];
                __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): ftop must not stay pending
            }
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

    // Commutative per-node trace hash: no-return 64-bit atomic adds.  Terms for
    // the popped thread's node (nearly all of them) are summed in a register and
    // added once at the end of the iteration, after the step's loads were issued
    // (a load waits for every older store/atomic of the wave: vmcnt is in order).
    __device__ __forceinline__ void hash_atomic(uint32_t node, uint64_t v) {
        unsigned long long GAS* h = LP ? (unsigned long long GAS*)(gp(c.hash_g) + lane_of(node))
                                       : (unsigned long long GAS*)(gp(c.hash) + ix(node));
        __hip_atomic_fetch_add(h, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ __forceinline__ void hash_add(uint32_t node, uint64_t v) {
        if (node == hnode) hacc += v;
        else { STAT(K_HASH_IMM); hash_atomic(node, v); }
    }
    __device__ __forceinline__ void hash_flush() {
        if (hacc) { STAT(K_HASH_FLUSH); hash_atomic(hnode, hacc); }  // adding 0 is a no-op
        hacc = 0;
    }
    // every lane issues the atomic (adding 0 to its dummy word when it has no
    // term): one unconditional vector-memory op for the store tail's shape
    __device__ __forceinline__ void hash_flush_all() {
        const bool h = hacc != 0;
        unsigned long long GAS* p = h ? (LP ? (unsigned long long GAS*)(gp(c.hash_g) + lane_of(hnode))
                                            : (unsigned long long GAS*)(gp(c.hash) + ix(hnode)))
                                      : (unsigned long long GAS*)(gp(c.dummy) + TW_DUMMY_REC + r);
        __hip_atomic_fetch_add(p, (unsigned long long)hacc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        hacc = 0;
    }
    __device__ __forceinline__ void hash(uint32_t node, uint32_t kind, int64_t val) {
        hash_add(node, term(now, kind, val));
    }
    // LP mode: append a delivery record for another logical process
    __device__ __forceinline__ void emit(int64_t ta, int64_t payload, uint32_t link, uint32_t kind, uint32_t src,
                                         uint32_t dst, uint4 dh = make_uint4(0x80000000u, 0, 0, 0)) {
        if (c.dpar && c.win && !(dh.x >> 31) && dst - c.lp0 < c.R) {
            // a light local lane: straight into its inbox (buffer of the next
            // window), no tw_lp_pack pass.  The record is later than this window
            // (t >= window end: a send is at least the lookahead): instead of a
            // per-record atomic on the window's record minimum (one hot address)
            // the lane notes that it sent (DW_IB bit 31) and its epilogue lowers
            // the minimum to the window end once -- a bound below every such record
            const uint32_t lp = dst - c.lp0;
            const uint32_t par = (c.wid + 1u) & 1u;
            const uint32_t k = __hip_atomic_fetch_add(gp(c.inbox_n) + (size_t)par * c.R + lp, 1u, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
            if (k >= dh.z) {
                __hip_atomic_fetch_or(gp(c.lp_err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return;
            }
            const size_t base = c.ib_off ? ((size_t)dh.y << c.rep_lg) + (dst & ((1u << c.rep_lg) - 1u)) : (size_t)lp;
            uint4 GAS* q = gp(c.inbox) + ((size_t)par * c.ib_total + base + (size_t)k * ib_stride(c, false)) * 2;
            q[0] = make_uint4((uint32_t)ta, (uint32_t)((uint64_t)ta >> 32), (uint32_t)payload,
                              (uint32_t)((uint64_t)payload >> 32));
            q[1] = make_uint4(link, kind, src, dst);
            lp_list_next(c, lp);
            ds(DW_IB, dg(DW_IB) | 0x80000000u);
            return;
        }
        if (c.dpar && c.win && (dh.x >> 31) && dst - c.lp0 < c.R) {
            // a heavy local lane: straight into its inbox too (buffer 0, which
            // tw_lp_due reads at the next window's first tick, before any event
            // kernel of that window), with tw_lp_pack's bookkeeping: the next
            // window's heavy list on the first pending record, the mark, and
            // the window-minimum bound of the light path above
            const uint32_t lp = dst - c.lp0;
            const uint32_t k = __hip_atomic_fetch_add(gp(c.inbox_n) + lp, 1u, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
            if (k >= dh.z) {
                __hip_atomic_fetch_or(gp(c.lp_err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return;
            }
            const size_t base = c.ib_off ? ib_heavy_base(c, dh.y, dh.z, dst) : (size_t)lp;
            uint4 GAS* q = gp(c.inbox) + (base + (size_t)k * ib_stride(c, true)) * 2;
            q[0] = make_uint4((uint32_t)ta, (uint32_t)((uint64_t)ta >> 32), (uint32_t)payload,
                              (uint32_t)((uint64_t)payload >> 32));
            q[1] = make_uint4(link, kind, src, dst);
            if (k == 0) {
                const uint32_t l = (c.wid + 1u) & 1u;
                const uint32_t j = __hip_atomic_fetch_add(gp(c.heavy_n) + l, 1u, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
                if (j < c.R) gp(c.heavy)[(size_t)l * c.R + j] = lp;
                else __hip_atomic_fetch_or(gp(c.lp_err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            lp_list_next(c, lp);
            ds(DW_IB, dg(DW_IB) | 0x80000000u);
            return;
        }
        const uint32_t i = wave_append(gp(c.out_n), 1u);
        if (i >= c.out_cap) {
            __hip_atomic_fetch_or(gp(c.lp_err), 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        uint4 GAS* o = gp(c.outbox) + (size_t)i * 2;
        o[0] = make_uint4((uint32_t)ta, (uint32_t)((uint64_t)ta >> 32), (uint32_t)payload,
                          (uint32_t)((uint64_t)payload >> 32));
        o[1] = make_uint4(link, kind, src, dst);
    }
    // Batched LP: a fork onto another node of this replica.  The child is
    // queued at t on that node's lane (TimedT.hs:326-339) by the spawn record
    // pair this appends (tw_lp_pack hands it over; the lane creates the thread
    // at its next tick, before running anything later than t).
    __device__ __forceinline__ void emit_spawn(int64_t t, uint32_t pc, uint32_t dst, int64_t q0, int64_t q1,
                                               int64_t q2, int64_t q3) {
        const uint32_t i = wave_append(gp(c.out_n), 2u);
        if (i + 1 >= c.out_cap) {
            __hip_atomic_fetch_or(gp(c.lp_err), 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        uint4 GAS* o = gp(c.outbox) + (size_t)i * 2;
        o[0] = make_uint4((uint32_t)t, (uint32_t)((uint64_t)t >> 32), (uint32_t)q0, (uint32_t)((uint64_t)q0 >> 32));
        o[1] = make_uint4(pc, TW_SPAWN_KIND, 0u, dst);
        o[2] = make_uint4((uint32_t)q1, (uint32_t)((uint64_t)q1 >> 32), (uint32_t)q2, (uint32_t)((uint64_t)q2 >> 32));
        o[3] = make_uint4((uint32_t)q3, TW_SPAWN_CONT, (uint32_t)((uint64_t)q3 >> 32), dst);
    }
    // LP: pop the head of the due run.  The record becomes the deliverer's
    // phantom thread (its wake pop, counted by the sender) in a fresh slot,
    // exactly as if it had been queued at the window's start.
    __device__ __forceinline__ void due_pop(Th& th, uint32_t& slot, uint32_t sq) {
        const uint32_t hn = dg(DW_HN), h = hn & 0xFFFFu, n = hn >> 16;
        const size_t ib = dg(DW_IB) & 0x7FFFFFFFu, st = ib_stride(c, true);  // (a due run: a heavy lane's)
        const uint4 GAS* q = gp(c.due) + (ib + (size_t)h * st) * 2;
        const uint4 a = q[0], b = q[1];
        const uint4 nx = gp(c.due)[(ib + (size_t)(h + 1 < n ? h + 1 : h) * st) * 2];
        tw_vm_drain();
        ds(DW_HN, hn + 1);
        ds(DW_TL, nx.x);
        ds(DW_TH, nx.y);
        far_dirty = true;
        const uint32_t s = alloc_slot();
        const bool ok = s != 0xFFFFFFFFu;
        th.w0 = ((TW_PC_DELIVER_STUB + 1) & 0xFFFFu) | ((F_STARTED | F_PHANTOM) << FL_SHIFT);
        th.w1 = (c.lp0 + r) >> c.rep_lg;
        th.w2 = 0xFFFFFFFEu;      // never a throwTo target
        th.w3 = ok ? sq : sq + 1; // no slot (the lane has failed): a pop without effect
        th.f0 = th.f1 = 0;
        th.xl = b.w;  // the reply link (tw_lp_due), flagged by xh: DELIVER takes it and clears both
        th.xh = 1;
        th.r0 = (int64_t)(((uint64_t)a.w << 32) | a.z);  // payload
        th.r1 = b.x;                                     // link
        th.r2 = b.z;                                     // sending node
        th.r3 = b.y;                                     // kind
        live += ok ? 1u : 0u;
        slot = ok ? s : 0u;
    }

    // Create a thread queued at now (fork, TimedT.hs:326-339): its record is
    // left in `ch` for the store tail.  Returns its ref.
    // queue = false: the child is the very next pop and runs in place (step):
    // its queue entry's insertion counter value is taken, the entry itself and
    // the live count's +1 / -1 of its push and pop are left out
    __device__ __forceinline__ bool spawn(uint32_t pc, uint32_t node, int64_t q0, int64_t q1, int64_t q2, int64_t q3,
                                          int64_t& ref, Th& ch, uint32_t& cs_out, bool queue = true) {
        uint32_t s = alloc_slot();
        if (s == 0xFFFFFFFFu) return false;
        if (tidc == 0xFFFFFFFFu) { fail(TW_REP_ERR_COUNTER); return false; }  // getNextThreadId, TimedT.hs:288-289
        uint32_t tid = tidc++;
        ++d_th;
        ch.w0 = pc & 0xFFFFu;
        ch.w1 = node;
        ch.w2 = tid;
        ch.w3 = 0;
        ch.f0 = ch.f1 = ch.xl = ch.xh = 0;
        ch.r0 = q0; ch.r1 = q1; ch.r2 = q2; ch.r3 = q3;
        if (queue) enqueue(ch, s, now, true);
        else (void)next_seq(true);
        cs_out = s;
        ref = (int64_t)(((uint64_t)tid << 32) | s);
        return true;
    }

    // throwTo (TimedT.hs:357-368) for the lanes `thr` of an interpreter pass
    // (n: the instruction's count in the step): the target's event is
    // re-stamped to now, the first exception wins.  Only the victim's header
    // quad is read and written (pc, flags, exception code, tid, queued seq); a
    // fresh exception's value goes to the upper half of its frames quad with
    // one 8-B store.  The header comes from the quad stage_victims loaded at the
    // pop when this is the step's first or second instruction, else from HBM
    // here (drained in place on every path).
    __device__ __forceinline__ void throw_to(Th& self, uint32_t self_slot, uint32_t n, bool thr, int64_t ref,
                                            uint32_t code, int64_t val) {
        const uint32_t ts = (uint32_t)ref;
        const uint32_t tid = (uint32_t)((uint64_t)ref >> 32);
        bool go = thr && ts < c.S;
        if (go && ts == self_slot) {  // the running thread: its record lives in registers
            if (self.w2 == tid && th_exc(self) == 0) { th_set_exc(self, code); th_set_xval(self, val); q1d = true; }
            go = false;
        }
        uint32_t k = 2u;  // the staged quad holding this lane's victim header (2: none)
        if constexpr (HR) {
            if (__builtin_amdgcn_ballot_w64(go && n <= 3u)) {
                // (CW_VS: d_ev << 3 | the step's first pass count n0 << 2 | quads)
                const uint32_t vs = cg(CW_VS);
                const uint32_t j = n - 1u - ((vs >> 2) & 1u);  // 0, 1: the step's first / second pass
                const bool st = go && j < 2u && (vs >> 3) == d_ev && ((vs >> j) & 1u);
                k = st ? j : 2u;
            }
        }
        uint4 h = make_uint4(0u, 0u, 0xFFFFFFFFu, 0u);
        if (__builtin_amdgcn_ballot_w64(k < 2u)) {
            // every vector-memory op since the staging load is younger: the record
            // prefetch's four at least
            asm volatile("s_waitcnt vmcnt(4) ; tw:vic" ::: "memory");
            if (k < 2u) h = qq[k * WG];
        }
        if (__builtin_amdgcn_ballot_w64(go && k == 2u)) {
            if (go && k == 2u) h = hrec(ts)[0];
            tw_vm_drain();
        }
        if (!go || h.z != tid) return;  // dead (slot free or reused): the map entry is unobservable
        Th t;
        t.w0 = h.x; t.w1 = h.y; t.w2 = h.z; t.w3 = h.w;
        if (t.w3 != 0) {          // queued: wake to now with a fresh seq
            bool on_chip = (th_flags(t) & F_NEARQ) != 0;
            uint32_t s = next_seq();
            if (!(on_chip && near_rekey(t.w3, now, s, ts))) {
                on_chip = near_fits(now);
                if (on_chip) {
                    near_push(now, s, ts);
                } else if (!run_push(now, s, ts)) {
                    far_push(now, s, ts);
                    // (the heap's ancestor loads whose values go unused must not stay
                    // in flight into the next pass; the stores of every other path
                    // need no wait: a wave's later loads of the same words see them)
                    tw_vm_drain();
                }
            }
            if (on_chip) th_or_flags(t, F_NEARQ);
            else th_clr_flags(t, F_NEARQ);
            t.w3 = s;
        }
        const bool fresh = th_exc(t) == 0;
        if (fresh) th_set_exc(t, code);
        if (ts == pf_slot) pf_slot = 0xFFFFFFFFu;
        STAT(K_PUT_HBM);
        uint4 GAS* p = hrec(ts);
        p[0] = make_uint4(t.w0, t.w1, t.w2, t.w3);
        if (fresh)  // (xl, xh: the frames quad's upper half)
            *(uint2 GAS*)((uint32_t GAS*)(p + c.RQ) + 2) = make_uint2((uint32_t)val, (uint32_t)((uint64_t)val >> 32));
    }

    // A thread resumed at an unconditional JMP -- every `schedule`'s stub
    // (`wait spec >> jmp action`, program.py Code.schedule; MonadTimed.hs:162-163)
    // -- goes to the jump's target at the pop: the JMP counts as the step's
    // first instruction (n0 = 1) without an interpreter pass of its own.  The
    // resume pc's pop word (PW, pop_word: made in the launch prologue) holds the
    // pc to start at, n0 and the victim staging's throwTo flags, one LDS read.
    __device__ __forceinline__ uint32_t jump_at_pop(Th& th, bool run, uint32_t& pw) const {
        const uint32_t pc = th_pc(th);
        const bool ok = run && pc < c.n_insns;
        pw = PW[ok ? pc : c.n_insns];  // (entry n_insns: no flags)
        th.w0 = ok ? (th.w0 & 0xFFFF0000u) | (pw & 0xFFFFu) : th.w0;
        return ok ? (pw >> 16) & 1u : 0u;
    }

    // Victim prefetch (replica kernels).  A step that opens with throwTo -- C3's
    // kill pair `mapM_ killThread [r1, r2]` at 120 s, 4,096 per replica
    // (examples/token-ring/Main.hs:124-127) -- waited a full HBM round trip for
    // each victim's header in its interpreter pass.  The victims are known at
    // the pop (the refs sit in the popped record's registers), so their header
    // quads are loaded here, by LDS-DMA into the child-register quads (qq: free
    // until a spawning instruction later in the step), for the step's first two
    // instructions when they are throwTo.  Issued before the record prefetch,
    // so throw_to's counted vmcnt(4) proves they landed without waiting for
    // it.  CW_VS names this pop (d_ev: every counted pop and in-place child
    // changes it), the step's starting instruction count n0 and the staged quads.
    __device__ __forceinline__ void stage_victims(uint32_t slot, bool run, uint32_t n0, uint32_t pw) {
        const bool t0 = run && ((pw >> 17) & 1u);
        if (!__builtin_amdgcn_ballot_w64(t0)) return;
        const uint32_t v0 = (uint32_t)rf[((pw >> 19) & 3u) * WG];
        const uint32_t v1 = (uint32_t)rf[((pw >> 21) & 3u) * WG];
        const bool s0 = t0 && v0 < c.S && v0 != slot;
        const bool s1 = t0 && ((pw >> 18) & 1u) && v1 < c.S && v1 != slot && v1 != v0;
        // (readfirstlane: the m0 operand is an SGPR whatever register the value was kept in)
        const uint32_t qw = (uint32_t)__builtin_amdgcn_readfirstlane((int)(pfs_wave + qq_lds_offset<WG, NC, HR>()));
        asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off ; tw:vic" ::"v"(hrec(s0 ? v0 : 0u)),
                     "s"(qw) : "memory", "m0");
        if (__builtin_amdgcn_ballot_w64(s1))
            asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off ; tw:vic" ::"v"(hrec(s1 ? v1 : 0u)),
                         "s"(qw + WG * 16) : "memory", "m0");
        cs(CW_VS, (d_ev << 3) | (n0 << 2) | (s0 ? 1u : 0u) | (s1 ? 2u : 0u));
    }

    // Thread ends (END or uncaught exception): listener release, ref
    // invalidation, slot freed; the caller stores the header quad.
    __device__ __forceinline__ void rel_bind(const Th& th) {
        // an owned listener (token-ring `serve`) is released when its thread
        // dies: recorded with a store, no read (DELIVER compares the owner)
        if (th_flags(th) & F_OWNS) {
            gp(c.bind_rel)[bix(th.w1)] = th.w2;
            if constexpr (LP) ds(DW_BREL, th.w2);
        }
    }
    __device__ __forceinline__ void die_prep(Th& th, uint32_t slot) {
        rel_bind(th);
        th.w2 = 0xFFFFFFFFu;  // invalidate refs to this slot
        th.w3 = 0;
        free_slot(slot);
    }
    __device__ __forceinline__ void die(Th& th, uint32_t slot) {
        rel_bind(th);
        th.w2 = 0xFFFFFFFFu;  // invalidate refs to this slot
        th.w3 = 0;
        put_hdr(slot, th);
        free_slot(slot);
    }

    // Frames 2.. of the thread in `slot` (the handler stack beyond the record).
    __device__ __forceinline__ uint32_t GAS* fxp(uint32_t slot, uint32_t i) const {
        return (uint32_t GAS*)(gp(c.fx) + ((size_t)slot * c.R + r) * c.FXQ) + (i - 2);
    }
    __device__ __forceinline__ uint32_t frame(const Th& t, uint32_t slot, uint32_t i) const {
        if (i < 2) return i == 0 ? t.f0 : t.f1;
        const uint32_t f = *fxp(slot, i);
        tw_vm_drain();
        return f;
    }

    // Raise `code` in the running thread; true if a catch frame took it (pc set
    // to the handler, r0 = value, r3 = code in the register file).  Frames are
    // left innermost first, the way TimedT's ContException unwinds the
    // handler list (TimedT.hs:183-204, 263, 284); finally frames set their
    // timeout's done flag on the way (TimedT.hs:376).
    __device__ __forceinline__ bool unwind(Th& th, uint32_t slot, uint32_t code, int64_t val) {
        const uint32_t n = th_nfr(th);
        for (int i = (int)n - 1; i >= 0; --i) {
            const uint32_t f = frame(th, slot, (uint32_t)i);
            const uint32_t mask = f >> 16;
            if (mask == 0) {
                const uint32_t e = f & 0xFFFFu;
                if (e < c.T) gp(c.tmo_done)[ix(e)] = 1;
            } else if (mask & (1u << code)) {
                th_set_nfr(th, (uint32_t)i);
                th_set_pc(th, f & 0xFFFFu);
                rs(th, 0, val);
                rs(th, 3, (int64_t)code);
                return true;
            }
        }
        th_set_nfr(th, 0);
        if (th_flags(th) & F_MAIN) cs(CW_MAINEXC, code);
        die(th, slot);
        return false;
    }

    // TRACE record (tw_set_trace): appended in this replica's execution order
    __device__ __forceinline__ void trace_rec(uint32_t node, int32_t tag, int64_t val) {
        if constexpr (LP) return;  // (tw_set_trace refuses LP contexts: trace_cap is 0)
        const uint32_t n = cg(CW_TRN);
        cs(CW_TRN, n + 1);
        if (n < c.trace_cap) {
            uint4 GAS* q = gp(c.trace) + ((size_t)n * c.R + r) * 2;
            q[0] = make_uint4((uint32_t)now, (uint32_t)((uint64_t)now >> 32), node, (uint32_t)tag);
            q[1] = make_uint4((uint32_t)val, (uint32_t)((uint64_t)val >> 32), 0u, 0u);
        }
    }

    // ------------------------------------------------------------- interpreter
    __device__ __forceinline__ void pfail(bool cond, uint32_t st) {
        status = (cond && status == TW_REP_RUNNING) ? st : status;
    }
    // predicated cold-word store: idle lanes write a dummy word (no branch)
    __device__ __forceinline__ void csp(bool p, int w, uint32_t v) {
        if constexpr (CWR) cwr[w] = p ? v : cwr[w];
        else cw[(p ? w : CW_DUMMY) * WG] = v;  // idle lanes write a dummy word (no branch)
    }

    enum { T_NONE, T_YIELD, T_SPAWN, T_EXIT, T_STOP, T_DIED };
    // The step's per-lane loop state, shared by the interpreter's passes
    struct St {
        uint32_t pc, fin, n;
        bool running;
        int64_t yt;
    };

    // One interpreter pass: the instruction (uw, imm; op and uop flags fl of the
    // first running lane, lfl of this lane's own) for the lanes `at` it.
    __device__ __forceinline__ void pass(Th& th, uint32_t slot, St& s, bool at, uint32_t uw, int32_t imm, uint32_t op,
                                         uint32_t fl, uint32_t lfl) {
        uint32_t& pc = s.pc;
        bool& running = s.running;
        uint32_t& n = s.n;
        int64_t& yt = s.yt;
        uint32_t& fin = s.fin;
        const bool hot = !(fl & U_FX);
        n += at ? 1u : 0u;
        const bool capped = at && n > TW_STEP_CAP;  // TW_REP_ERR_INSN before executing it
        const bool me = at && !capped;
        const uint32_t a = (uw >> 8) & 3u, b = uw >> 16;
        STAT(K_INSN);
        const int64_t ra = rg(th, a);
        const int64_t rb = rg(th, (b & 3u));
        uint32_t tc = T_NONE;     // per lane: terminal action of this op
        uint32_t tgt = pc + 1;    // per lane: next pc
        bool wr = false;          // uniform: the op writes r[a]
        bool wm = me;             // per lane: ... in this lane
        int64_t wv = 0;
        bool thr_any = false, thr = false;  // throwTo after the op (THROW_TO, TMO_FIRE)
        int64_t tref = 0, tval = 0;
        uint32_t tcode = 0;
        // ---- hot classes: register result, table load, trace, jump, yield/exit/
        // fork.  When every lane of the pass holds the same uop (lock-step
        // lanes) the classes are wave-uniform scalar branches on the first
        // lane's uop; otherwise each lane evaluates its own uop and a class
        // runs when some lane needs it (ballot).
        auto hot_body = [&](auto uni, uint32_t f) {
            constexpr bool U = decltype(uni)::value;
            auto need = [&](bool lane_cond) -> bool {
                if constexpr (U) return lane_cond;
                else return __builtin_amdgcn_ballot_w64(me && lane_cond) != 0;
            };
            const uint32_t ak = U_ALU(f), tk = U_TK(f), jm = U_JM(f), ld = U_LD(f);
            bool lw = false;
            if (need(ak != A_NONE)) {
                const int64_t i64 = imm;
                int64_t kv = K[ak == A_K ? imm : 0];
                int64_t v = i64;
                v = ak == A_ADDI ? ra + i64 : v;
                v = ak == A_MULI ? ra * i64 : v;
                v = ak == A_MOV ? rb : v;
                v = ak == A_ADD ? ra + rb : v;
                v = ak == A_SUB ? ra - rb : v;
                v = ak == A_NOW ? now : v;
                v = ak == A_NODE ? (int64_t)th.w1 : v;
                v = ak == A_TID ? (int64_t)(((uint64_t)th.w2 << 32) | slot) : v;
                // per-lane mode: keep the pool read unconditional (the compiler would
                // otherwise sink it into a divergent region)
                if constexpr (!U) asm volatile("" : "+v"(kv));
                v = ak == A_K ? kv : v;
                wr = true;
                lw = ak != A_NONE;
                wv = v;
            }
            if (need(ld != LD_NONE)) {
                // NLOAD r[a] <- var b of this node; LINK r[a] <- out_off[node] + imm;
                // RLINK r[a] <- link_rev[r[b]] (an out-of-range link stops the replica)
                const bool nv = me && ld == LD_NV, ol = me && ld == LD_OUT, rl = me && ld == LD_RL;
                const bool bad = rl && (uint64_t)rb >= c.L;
                pfail(bad, TW_REP_ERR_INSN);
                tc = bad ? (uint32_t)T_STOP : tc;
                int64_t v = wv;
                if (need(ld == LD_NV)) {
                    const int64_t x = gp(c.nvars)[nix(nv ? th.w1 : 0u, b & 3)];
                    v = nv ? x : v;
                }
                bool cached = false;
                if constexpr (LP) {
                    // every lane's LINK / RLINK answered from the lane's cache: no load, no wait
                    const bool miss = rl && (uint32_t)rb != rlc_link;
                    if (need(ld == LD_OUT || ld == LD_RL) && !__builtin_amdgcn_ballot_w64(miss) &&
                        !__builtin_amdgcn_ballot_w64(me && ld == LD_NV)) {
                        v = ol ? (int64_t)oo + imm : (rl ? (int64_t)rlc_rev : v);
                        cached = true;
                    }
                }
                if (!cached && need(ld == LD_OUT || ld == LD_RL)) {
                    const uint32_t GAS* tb = ol ? gp(c.out_off) : gp(c.link_rev);
                    const uint32_t x = tb[ol ? (size_t)th.w1 : (rl && !bad ? (size_t)rb : 0)];
                    v = ol ? (int64_t)x + imm : (rl ? (int64_t)x : v);
                }
                if (!cached) tw_vm_drain();
                wr = true;
                lw = lw || ((nv || ol || rl) && !bad);
                wv = v;
            }
            wm = me && lw;
            if (need((f & U_NS) != 0)) {  // fused NSTORE of the ALU result
                if (me && (f & U_NS)) gp(c.nvars)[nix(th.w1, b & 3u)] = wv;
            }
            if (need((f & U_TR) != 0)) {  // the popped node's term joins hacc
                hacc += (me && (f & U_TR)) ? term(now, TW_KIND_TRACE | ((uint32_t)imm & 0xFFFFu), ra) : 0ull;
                if (c.trace_cap && me && (f & U_TR)) trace_rec(th.w1, imm, ra);
            }
            if (need((f & U_TR2) != 0)) {  // fused second TRACE
                const bool t2l = me && (f & U_TR2);
                const int64_t r2 = rg(th, ((b >> 13) & 3u));
                hacc += t2l ? term(now, TW_KIND_TRACE | (b & 0x1FFFu), r2) : 0ull;
                if (c.trace_cap && t2l) trace_rec(th.w1, (int32_t)(b & 0x1FFFu), r2);
            }
            if (need((f & U_P2) != 0)) tgt = (f & U_P2) ? pc + 2 : tgt;
            if (need(jm != JM_NONE)) {
                const int64_t b16 = (int64_t)(int16_t)b;
                const uint32_t ci = (ra == rb ? 1u : 0u) | (ra < rb ? 2u : 0u) | (ra == b16 ? 4u : 0u);
                tgt = ((jm >> ci) & 1u) ? (uint32_t)imm : tgt;
            }
            if (need(tk != TK_NONE)) {
                tc = tk == TK_EXIT ? (uint32_t)T_EXIT : tc;
                if (need(tk == TK_FORK)) {
                    const bool fk = tk == TK_FORK;
                    const uint32_t node = b == 0xFFFFu ? th.w1 : (uint32_t)rb;
                    const bool bad = fk && (LP ? (c.lpb ? node >= c.Ntot : node != th.w1) : node >= c.N);
                    pfail(me && bad, TW_REP_ERR_INSN);
                    tc = fk ? (bad ? (uint32_t)T_STOP : (uint32_t)T_SPAWN) : tc;
                    const bool p = me && fk && !bad;
                    csp(p, CW_CSP, csp_word((uint32_t)imm, a, 2u));  // the child's registers are the parent's
                    csp(p, CW_CNODE, node);
                    if constexpr (LP) {
                        // batched LP, a fork onto another node of the replica
                        // (TimedT.hs:326-342): the child goes out as a spawn record
                        // right here, with the registers it captures now, and the
                        // parent's `wait (for 1 mcs)` becomes an ordinary yield --
                        // which the inline continuation below resumes in this pass
                        // when nothing on the node is due before it (a main thread
                        // forking every node of the scenario runs its loop without a
                        // queue round trip per fork)
                        const bool xs = p && c.lpb && node != th.w1;
                        if (__builtin_amdgcn_ballot_w64(xs)) {
                            bool ph1 = false;
                            if (xs && c.phase) {
                                ph1 = gp(c.phase)[th.w1] != 0;  // (not from a phase-1 node)
                                tw_vm_drain();
                            }
                            const bool go = xs && !ph1;
                            pfail(xs && ph1, TW_REP_ERR_INSN);
                            tc = (xs && ph1) ? (uint32_t)T_STOP : tc;
                            if (go) {
                                emit_spawn(now, (uint32_t)imm, lane_of(node), rg(th, 0), rg(th, 1), rg(th, 2), rg(th, 3));
                                rs(th, a, -1);  // the ref is opaque (refs name engine slots)
                            }
                            tc = go ? (uint32_t)T_YIELD : tc;
                            yt = go ? now + 1 : yt;
                            if (TW_LP_FORKN && __builtin_amdgcn_ballot_w64(go && (lfl & U_FL)))
                                if (go && (lfl & U_FL)) fork_loop(th, n, pc, (uint32_t)imm, a, b, tgt, tc, yt);
                        }
                    }
                }
                const bool wt = tk == TK_WREL || tk == TK_WABS || tk == TK_WREG;
                if (need(wt)) {
                    int64_t kt = K[(wt && tk != TK_WREG) ? imm : 0];
                    int64_t w = now + (ra > 0 ? ra : 0);               // wait (for r[a])
                    if constexpr (!U) asm volatile("" : "+v"(kt));
                    w = tk == TK_WREL ? now + kt : w;                    // wait (for K)
                    w = tk == TK_WABS ? (kt > now ? kt : now) : w;       // wait (till K)
                    yt = (me && wt) ? w : yt;
                    tc = wt ? (uint32_t)T_YIELD : tc;
                }
            }
        };
        if (hot) {
            if constexpr (PL) {
                if (__builtin_expect(__builtin_amdgcn_ballot_w64(at && ((lfl ^ fl) & (FOLDJ ? ~U_FOLD : ~0u)) != 0) == 0, 1))
                    hot_body(BoolC<true>{}, fl);
                else
                    hot_body(BoolC<false>{}, lfl);
            } else {
                hot_body(BoolC<true>{}, fl);
            }
        }
        if ((fl & U_FX) != 0) {
        // the rare ops
        switch (op) {
        case TW_OP_THROW_TO: {
            thr_any = true; thr = me;
            tref = ra; tcode = b & 0xFFu; tval = rg(th, ((b >> 8) & 3u));
            break;
        }
        case TW_OP_THROW: {
            if (me) {
                th_set_pc(th, pc + 1);
                if (unwind(th, slot, b & 0xFFu, rg(th, ((b >> 8) & 3u)))) tgt = th_pc(th);
                else tc = T_DIED;  // died: record stored
            }
            break;
        }
        case TW_OP_CATCH:
        case TW_OP_TMO_PUSH: {
            const uint32_t nf = th_nfr(th);
            const bool bad = nf >= c.max_frames;
            pfail(me && bad, TW_REP_ERR_FRAMES);
            tc = bad ? T_STOP : T_NONE;
            const uint32_t fv = op == TW_OP_CATCH ? (b << 16) | ((uint32_t)imm & 0xFFFFu) : (uint32_t)ra & 0xFFFFu;
            const bool ok = me && !bad;
            th.f0 = (ok && nf == 0) ? fv : th.f0;
            th.f1 = (ok && nf == 1) ? fv : th.f1;
            q1d = q1d || (ok && nf < 2);
            if (ok && nf >= 2) *fxp(slot, nf) = fv;  // deeper frames: the overflow area
            th.w0 = ok ? (th.w0 & ~(15u << 16)) | ((nf + 1) << 16) : th.w0;
            break;
        }
        case TW_OP_UNCATCH: {
            const uint32_t nf = th_nfr(th);
            const bool bad = nf == 0 || (frame(th, slot, nf > 0 && me ? nf - 1 : 0) >> 16) == 0;
            pfail(me && bad, TW_REP_ERR_INSN);
            tc = bad ? T_STOP : T_NONE;
            th.w0 = (me && !bad) ? (th.w0 & ~(15u << 16)) | ((nf - 1) << 16) : th.w0;
            break;
        }
        case TW_OP_MODI: {
            const int64_t m = ra % (int64_t)imm;
            wr = true;
            wv = m < 0 ? m + imm : m;
            break;
        }
        case TW_OP_NSTORE: {
            if (me) gp(c.nvars)[nix(th.w1, b & 3)] = ra;
            break;
        }
        case TW_OP_NLOADX:
        case TW_OP_NSTOREX: {
            const uint64_t node = (uint64_t)rg(th, ((b >> 8) & 3u));
            const bool bad = LP ? node != th.w1 : node >= c.N;
            pfail(me && bad, TW_REP_ERR_INSN);
            tc = bad ? T_STOP : T_NONE;
            const bool ok = me && !bad;
            int64_t GAS* v = &gp(c.nvars)[nix(ok ? (uint32_t)node : 0u, b & 3)];
            if (op == TW_OP_NLOADX) {
                wr = true; wm = ok; wv = *v;
            } else if (ok) {
                *v = ra;
            }
            tw_vm_drain();
            break;
        }
        case TW_OP_SEND: {  // schedule (after d) (deliver ..) unless the link drops it
            STIME(tsd0);
            wr = true;
            wm = false;
            if (me) {
                // fused LINK / RLINK (TW_SEND_VIA_*): the pair's first instruction
                // here, the pass continues past the pair's SEND (LP: the lane's
                // out-link base and last reply link are cached)
                uint64_t link = (uint64_t)ra;
                bool lbad = false;
                const bool fz = (b & (TW_SEND_VIA_LINK | TW_SEND_VIA_RLINK)) != 0;
                if (b & TW_SEND_VIA_LINK) {
                    link = (uint64_t)((int64_t)(LP ? oo : gp(c.out_off)[th.w1]) + imm);
                } else if (b & TW_SEND_VIA_RLINK) {
                    const uint64_t rin = (uint64_t)rg(th, ((b >> 12) & 3u));
                    lbad = rin >= c.L;
                    if (!lbad) link = (LP && (uint32_t)rin == rlc_link) ? rlc_rev : gp(c.link_rev)[rin];
                }
                wm = fz && !lbad;
                wv = (int64_t)link;
                tgt = fz ? pc + 2 : tgt;
                if (lbad || link >= c.L) {
                    fail(TW_REP_ERR_INSN);
                    tc = T_STOP;
                } else {
                    const uint32_t kind = b & 0xFFu;
                    const uint32_t pr = (b >> 8) & 3u;
                    const int64_t payload = (fz && pr == a) ? (int64_t)link : rg(th, pr);
                    // the link's ordinal and (LP) its destination entry: independent
                    // loads in flight together, one wait
                    // (a one-deep table -- one delay per link, every scenario but
                    // record-replay -- needs no ordinal: its entry is known now)
                    uint32_t ord = 0;
                    if (c.D > 1) {
                        ord = gp(c.link_ord)[lix(link)];
                        gp(c.link_ord)[lix(link)] = ord + 1;
                    }
                    uint4 dh = make_uint4(0x80000000u, 0, 0, 0);
                    if (LP) dh = gp(c.link_dsth)[link];  // destination | heavy, its inbox
                    const uint32_t e = c.link_table ? gp(c.link_table)[tix(link, ord)] : 0u;
                    if (e & TW_LINK_DROP) {
                        cinc(CW_DR);
                        hash(th.w1, TW_KIND_DROP | kind, payload);
                    } else if (LP) {
                        // the deliverer `schedule (after d) deliver` is accounted here (start pop
                        // at now, wake pop at now+d, both at this node) and its delivery travels
                        // as a record: the receiver checks its binding at now+d
                        const int64_t dly = (int64_t)(e & 0x7FFFFFFFu) + tx_us(c, link, kind);
                        // shorter than the lookahead: only from a phase-0 node into a
                        // phase-1 node (delivered in this window's phase 1)
                        if (dly < c.lookahead &&
                            !(c.phase && gp(c.phase)[th.w1] == 0 && gp(c.phase)[gp(c.link_dst)[link]] == 1)) {
                            fail(TW_REP_ERR_INSN);
                            tc = T_STOP;
                        } else {
                            const int64_t ta = now + dly;
                            hash_add(th.w1, term0(now, TW_KIND_RESUME | TW_PC_DELIVER_STUB) +
                                                term0(ta, TW_KIND_RESUME | (TW_PC_DELIVER_STUB + 1)));
                            d_ev += 2;
                            ++d_th;
                            final_t = ta > final_t ? ta : final_t;
                            emit(ta, payload, (uint32_t)link, kind, th.w1, lane_of(dh.x & 0x7FFFFFFFu), dh);
                            yt = now + 1;
                            tc = T_YIELD;
                        }
                    } else {
                        cs(CW_CSP, csp_word(TW_PC_DELIVER_STUB, 4u, 0u)); cs(CW_CNODE, th.w1);
                        qset(payload, (int64_t)link, (int64_t)(e & 0x7FFFFFFFu) + tx_us(c, link, kind), (int64_t)kind);
                        tc = T_SPAWN;
                    }
                }
            }
            // (LP: every load above was consumed; what is left in flight are the
            // record's stores, which the next pop's counted wait covers)
            if (!LP) tw_vm_drain();
            STIME(tsd1);
            STADD(K_CYC_SEND, tsd1 - tsd0);
            break;
        }
        case TW_OP_DELIVER: {  // listener dispatch, ForkStrategy fork_ (MonadDialog.hs:232-256,317)
            STIME(tdl0);
            if (me) {
                const int64_t r0 = rg(th, 0), r1 = rg(th, 1), r2 = rg(th, 2), r3 = rg(th, 3);
                const uint64_t link = (uint64_t)r1;
                const uint32_t kind = (uint32_t)r3;
                // LP: the record reached its destination's lane, whose binding
                // words are cached in LDS; the handler table is staged in LDS
                const uint32_t dst = LP ? th.w1 : gp(c.link_dst)[link];
                const uint32_t set0 = LP ? dg(DW_BSET) : gp(c.bind)[bix(dst)];
                const uint32_t own = LP ? dg(DW_BOWN) : gp(c.bind_own)[bix(dst)];
                const uint32_t rel = LP ? dg(DW_BREL) : gp(c.bind_rel)[bix(dst)];
                if (LP) {
                    // the reply link a handler's RLINK asks for: a due-run record
                    // brought it (xh set); a light-inbox one loads it (drained in
                    // place, so a pass where no lane loads waits for nothing)
                    uint32_t rv = th.xl;
                    if (!th.xh) {
                        rv = gp(c.link_rev)[link];
                        tw_vm_drain();
                    }
                    th.xl = th.xh = 0;
                    rlc_rev = rv;
                    rlc_link = (uint32_t)link;
                }
                const uint32_t set = own == rel ? 0u : set0;  // owner died: released
                uint32_t lpc = TW_PC_NONE;
                if (set && kind < c.n_kinds) lpc = LPC[(size_t)(set - 1) * c.n_kinds + kind];
                if (lpc == TW_PC_NONE) {
                    cinc(CW_UD);
                    hash(dst, TW_KIND_UNDELIV | kind, r0);
                    if (LP) tc = T_EXIT;  // the phantom deliverer ends here
                } else if (lpc & TW_LPC_INLINE) {
                    // ForkStrategy `const id` (MonadDialog.hs:114-117): the handler runs
                    // in this thread on the destination node -- its terms go to dst
                    cinc(CW_DL);
                    hash(dst, TW_KIND_RECV | kind, r0);
                    hash_flush();
                    rs(th, 0, r0); rs(th, 1, (int64_t)link); rs(th, 2, LP ? r2 : (int64_t)th.w1);
                    rs(th, 3, (int64_t)kind);
                    hnode = dst;
                    th.w1 = dst;
                    // LP: the phantom deliverer becomes the handler thread, whose
                    // later pops are ordinary (counted and hashed) pops
                    th_clr_flags(th, F_PHANTOM);
                    tgt = lpc & ~TW_LPC_INLINE;
                } else if (LP && d_ev + 2 < ev_room && tidc != 0xFFFFFFFFu && seq != 0xFFFFFFFFu &&
                           queue_after(now)) {
                    // LP, ForkStrategy fork_ (MonadDialog.hs:317) when every queued event
                    // is later than now: the forked handler is the very next pop
                    // (TimedT.hs:326-342, 242), so this lane runs it in place.  As in
                    // the terminal's LP deliver fork, the deliverer's resume at now+1
                    // is accounted at the sending node; the handler's creation (thread
                    // id, insertion counter) and first pop (count, trace term) here.
                    cinc(CW_DL);
                    hash(dst, TW_KIND_RECV | kind, r0);
                    hash_add((uint32_t)r2, term0(now + 1, TW_KIND_RESUME | (TW_PC_DELIVER_STUB + 2)));
                    hash_add(dst, term0(now, TW_KIND_RESUME | (lpc & 0xFFFFu)));
                    d_ev += 2;
                    final_t = now + 1 > final_t ? now + 1 : final_t;
                    th.w2 = tidc++;
                    ++d_th;
                    (void)next_seq();
                    rs(th, 0, r0); rs(th, 1, (int64_t)link); rs(th, 2, r2); rs(th, 3, (int64_t)kind);
                    th_clr_flags(th, F_PHANTOM);
                    n = 0;  // TW_STEP_CAP counts per pop
                    tgt = lpc;
                } else {
                    cinc(CW_DL);
                    hash(dst, TW_KIND_RECV | kind, r0);
                    cs(CW_CSP, csp_word(lpc, 4u, LP ? 1u : 0u)); cs(CW_CNODE, dst);
                    qset(r0, (int64_t)link, LP ? r2 : (int64_t)th.w1, (int64_t)kind);
                    tc = T_SPAWN;
                }
            }
            if (!LP) tw_vm_drain();  // (LP: its one load drained in place)
            STIME(tdl1);
            STADD(K_CYC_DELIV, tdl1 - tdl0);
            break;
        }
        case TW_OP_LISTEN: {
            const bool bad = (uint32_t)imm >= c.n_sets;
            pfail(me && bad, TW_REP_ERR_INSN);
            tc = bad ? T_STOP : T_NONE;
            if (me && !bad) {
                gp(c.bind)[bix(th.w1)] = (uint32_t)imm + 1;
                gp(c.bind_own)[bix(th.w1)] = b ? th.w2 : 0xFFFFFFFFu;
                if constexpr (LP) {
                    ds(DW_BSET, (uint32_t)imm + 1);
                    ds(DW_BOWN, b ? th.w2 : 0xFFFFFFFFu);
                }
            }
            th.w0 = (me && !bad && b) ? th.w0 | (F_OWNS << FL_SHIFT) : th.w0;
            break;
        }
        case TW_OP_UNLISTEN: {
            if (me) {
                gp(c.bind)[bix(th.w1)] = 0;
                gp(c.bind_own)[bix(th.w1)] = 0xFFFFFFFFu;
                if constexpr (LP) {
                    ds(DW_BSET, 0);
                    ds(DW_BOWN, 0xFFFFFFFFu);
                }
            }
            break;
        }
        case TW_OP_TMO_BEGIN: {  // schedule (after t) watchdog (TimedT.hs:373-375)
            if (me) {
                const uint32_t tmo = cg(CW_TMO);
                if (tmo >= c.T) {
                    fail(TW_REP_ERR_INSN);
                    tc = T_STOP;
                } else {
                    cs(CW_TMO, tmo + 1);
                    gp(c.tmo_done)[ix(tmo)] = 0;
                    rs(th, a, tmo);
                    cs(CW_CSP, csp_word(TW_PC_WATCHDOG_STUB, 4u, 0u)); cs(CW_CNODE, th.w1);
                    qset((int64_t)(((uint64_t)th.w2 << 32) | slot), (int64_t)tmo, K[imm], 0);
                    tc = T_SPAWN;
                }
            }
            break;
        }
        case TW_OP_TMO_END: {
            if (me) {
                const uint32_t nf = th_nfr(th);
                const uint32_t fr = nf ? frame(th, slot, nf - 1) : 0u;
                if (nf == 0 || (fr >> 16) != 0) {
                    fail(TW_REP_ERR_INSN);
                    tc = T_STOP;
                } else {
                    const uint32_t ep = fr & 0xFFFFu;
                    th_set_nfr(th, nf - 1);
                    if (ep < c.T) gp(c.tmo_done)[ix(ep)] = 1;
                }
            }
            break;
        }
        case TW_OP_TMO_FIRE: {
            const uint64_t e = (uint64_t)rg(th, 1);
            const bool ok = me && e < c.T;
            thr_any = true;
            thr = ok && !gp(c.tmo_done)[ix(ok ? e : 0)];
            tref = rg(th, 0); tcode = TW_EXC_TIMEOUT; tval = 0;
            tw_vm_drain();
            break;
        }
        default: {  // an invalid opcode
            pfail(me, TW_REP_ERR_INSN);
            tc = T_STOP;
            break;
        }
        }
        }  // U_FX
        if (wr) rs(th, a, wm ? wv : ra);
        (void)lfl;
        if (thr_any) throw_to(th, slot, n, thr, tref, tcode, tval);
        // END folded into this pass: a lane whose next instruction is END
        // (U_NE / U_NE2 / U_JE) ends here, with END's count and pc, instead of
        // in a pass of its own -- launchNode's last END after its `when`
        // (examples/token-ring/Main.hs:125-131), the kill pair's after its throws
        if (FOLDJ && __builtin_amdgcn_ballot_w64(me && (lfl & U_FOLD) != 0)) {
          if constexpr (FOLD) {
            const bool fe = me && tc == T_NONE && status == TW_REP_RUNNING && n < TW_STEP_CAP &&
                            (((lfl & U_NE) && tgt == pc + 1u) || ((lfl & U_NE2) && tgt == pc + 2u) ||
                             ((lfl & U_JE) && tgt == (uint32_t)imm));
            n += fe ? 1u : 0u;
            tgt = fe ? tgt + 1u : tgt;
            tc = fe ? (uint32_t)T_EXIT : tc;
            const bool fw = me && tc == T_NONE && status == TW_REP_RUNNING && n < TW_STEP_CAP && (lfl & U_NW) &&
                            tgt == pc + 1u;
            if (__builtin_amdgcn_ballot_w64(fw)) {  // the wait's pass: its count, yield time and resume pc
                const uint2 wi = P[fw ? pc + 1u : 0u];
                const int64_t kt = K[fw ? wi.y : 0u];
                const int64_t w = (wi.x & 0xFFu) == TW_OP_WAIT_ABS ? (kt > now ? kt : now) : now + kt;
                n += fw ? 1u : 0u;
                yt = fw ? w : yt;
                tgt = fw ? pc + 2u : tgt;
                tc = fw ? (uint32_t)T_YIELD : tc;
            }
          }
            const bool fj = me && tc == T_NONE && status == TW_REP_RUNNING && n < TW_STEP_CAP && (lfl & U_NJ) &&
                            tgt == pc + 1u;
            if (__builtin_amdgcn_ballot_w64(fj)) {  // the jump's pass, on the registers as this pass left them
                const uint32_t jp = fj ? pc + 1u : 0u;
                const uint2 ji = P[jp];
                const uint32_t jm = U_JM(PU[jp]), jb = ji.x >> 16;
                const int64_t ja = rg(th, (ji.x >> 8) & 3u), jr = rg(th, jb & 3u);
                const uint32_t ci = (ja == jr ? 1u : 0u) | (ja < jr ? 2u : 0u) | (ja == (int64_t)(int16_t)jb ? 4u : 0u);
                const bool tk = (jm >> ci) & 1u;
                n += fj ? 1u : 0u;
                tgt = fj ? (tk ? ji.y : pc + 2u) : tgt;
                // ... and the END it lands on (`when` falling through to the end)
                const uint32_t jf = PU[jp];
                const bool je = fj && n < TW_STEP_CAP && (tk ? (jf & U_JE) != 0 : (jf & U_NE) != 0);
                n += je ? 1u : 0u;
                tgt = je ? tgt + 1u : tgt;
                tc = je ? (uint32_t)T_EXIT : tc;
            }
        }
        // per-lane epilogue of the pass
        pc = me ? tgt : pc;
        pfail(capped, TW_REP_ERR_INSN);
        const bool oob = tc == T_NONE && pc >= c.n_insns;
        pfail(me && oob, TW_REP_ERR_INSN);
        tc = capped ? (uint32_t)T_STOP : tc;
        tc = (tc == T_NONE && (status != TW_REP_RUNNING || oob)) ? (uint32_t)T_STOP : tc;
        if constexpr (LP) {
            // Inline continuation: a thread that yields to a time before every
            // event in its node's queue is the next pop (PQ.minView,
            // TimedT.hs:242), so it resumes here -- the pop's count, clock,
            // insertion-counter step and trace term as if it had been queued
            // and popped, without the queue round trip or a loop iteration.
            // (An LP node runs a few such yields per window -- every send
            // yields 1 µs -- and a wave waits for its busiest lane.)
            const bool y = me && tc == T_YIELD && !(th_flags(th) & F_PHANTOM) && status == TW_REP_RUNNING &&
                           seq != 0xFFFFFFFFu;
            if (__builtin_amdgcn_ballot_w64(y)) {
                if (far_dirty) far_min();
                const uint32_t sn = c.tie_mode ? seq_key(c.tie_mode, seq + 1) : seq + 1;
                bool has = near_n != 0;
                int64_t qt = nbase + (int64_t)(nrk >> 32);
                uint32_t qs = (uint32_t)nrk;
                const bool uf = fsrc >= 0 && (!has || tless(fmt, fms, qt, qs));
                qt = uf ? fmt : qt;
                qs = uf ? fms : qs;
                has = has || fsrc >= 0;
                const bool inl = y && yt <= t_end && d_ev < ev_room && (!has || tless(yt, sn, qt, qs));
                if (inl) {
                    STAT(K_POP);
                    ++seq;                       // the seq its queue entry would have taken
                    now = yt;                    // curTime .= timestamp
                    ++d_ev;
                    final_t = yt > final_t ? yt : final_t;
                    hacc += term0(yt, TW_KIND_RESUME | (pc & 0xFFFFu));
                    n = 0;                       // TW_STEP_CAP counts per pop
                    tc = T_NONE;
                    if (now - nbase > (int64_t)0x7FFFFFFF) near_rebase(now);
                    // the resumed instruction is END (a handler's last send, a
                    // gossip node's last forward): the thread ends in this pass
                    // instead of one more -- END's count, pc and exit as its pass
                    if (pc < c.n_insns && (P[pc].x & 0xFFu) == TW_OP_END) {
                        n = 1;
                        pc = pc + 1;
                        tc = T_EXIT;
                    }
                }
            }
        }
        fin = at ? tc : fin;
        running = running && !(at && tc != T_NONE);
    }
    // A counted loop of forks onto other nodes in one pass (LP kernels, round
    // 6: U_FL).  `forM_ [1..N] $ fork (launchNode ..)` (examples/token-ring/
    // Main.hs:65-68) lowers to `L: FORK a, pc, node r[b] ; ADDI x, k ; J* .., L`,
    // and in batched LP each fork is a spawn record plus the parent's 1-µs
    // yield, which the inline continuation resumes when nothing on the lane is
    // due first: two passes per fork (FOLDJ), ≈ 3 µs per fork on main's lane,
    // the chain of C3's start-up windows at 8,192 replicas per GPU (DESIGN
    // §3g).  Called after the pass emitted the first spawn, this runs the
    // loop's iterations as those passes would, one after the other: the
    // inline continuation of the yield at now + 1 (the epilogue's conditions,
    // count, clock, insertion-counter step and resume term; n restarts), the
    // ADDI, the jump (their counts), and while the jump goes back, the next
    // fork's spawn (its node checked first; a bad one is left to the next
    // pass at that pc, which fails it as it always has).  It stops where a
    // pass would leave the step or the loop: the yield not resumable (the
    // window's end, a queued event first, the event budget) -- the thread
    // yields at now + 1 from here -- or the jump falling through.
    __device__ __forceinline__ void fork_loop(Th& th, uint32_t& n, uint32_t pc, uint32_t imm, uint32_t a, uint32_t b,
                                           uint32_t& tgt, uint32_t& tc, int64_t& yt) {
        const uint2 ia = P[pc + 1u], ij = P[pc + 2u];
        const uint32_t x = (ia.x >> 8) & 3u, ja = (ij.x >> 8) & 3u, jb16 = ij.x >> 16;
        const uint32_t jm = U_JM(uop_of(ij.x & 0xFFu));
        for (;;) {
            // the parent's `wait (for 1 mcs)`, resumed inline (the pass epilogue's rule)
            if (status != TW_REP_RUNNING || seq == 0xFFFFFFFFu) break;
            if (far_dirty) far_min();
            const int64_t y = now + 1;
            const uint32_t sn = c.tie_mode ? seq_key(c.tie_mode, seq + 1) : seq + 1;
            bool has = near_n != 0;
            int64_t qt = nbase + (int64_t)(nrk >> 32);
            uint32_t qs = (uint32_t)nrk;
            const bool uf = fsrc >= 0 && (!has || tless(fmt, fms, qt, qs));
            qt = uf ? fmt : qt;
            qs = uf ? fms : qs;
            has = has || fsrc >= 0;
            if (!(y <= t_end && d_ev < ev_room && (!has || tless(y, sn, qt, qs)))) break;
            STAT(K_POP);
            ++seq;
            now = y;
            ++d_ev;
            final_t = y > final_t ? y : final_t;
            hacc += term0(y, TW_KIND_RESUME | ((pc + 1u) & 0xFFFFu));
            if (now - nbase > (int64_t)0x7FFFFFFF) near_rebase(now);
            // ADDI x, k ; J* (n restarted at the resume: two counts, never near the cap)
            rs(th, x, rg(th, x) + (int64_t)(int32_t)ia.y);
            const int64_t va = rg(th, ja), vb = rg(th, jb16 & 3u);
            const uint32_t ci = (va == vb ? 1u : 0u) | (va < vb ? 2u : 0u) | (va == (int64_t)(int16_t)jb16 ? 4u : 0u);
            n = 2;
            if (!((jm >> ci) & 1u)) {  // the loop ends: the pass goes on after the jump
                tc = T_NONE;
                tgt = pc + 3u;
                return;
            }
            // the next fork: its node checked as the pass checks it
            const uint32_t node = (uint32_t)rg(th, b & 3u);
            if (node >= c.Ntot || node == th.w1) {  // (a bad or own node: the next pass at pc)
                tc = T_NONE;
                tgt = pc;
                return;
            }
            n = 3;
            emit_spawn(now, imm, lane_of(node), rg(th, 0), rg(th, 1), rg(th, 2), rg(th, 3));
            rs(th, a, -1);
        }
        tc = T_YIELD;
        yt = now + 1;
        tgt = pc + 1u;
    }

    // Lock-step fast path (round 6, the run geometries: TW_FAST).  When every
    // running lane of the wave is at the same pc -- the replicas of one
    // scenario step through the same code, e.g. C3's start-up: main's `forM_
    // fork launchNode`, launchNode's forks, the worker's `catch ; sleepForever`,
    // the server's `listen ; sleepForever` (examples/token-ring/Main.hs:
    // 65-68,104-135) -- the instruction is one scalar word: it is read once
    // (an LDS broadcast) and decoded in SGPRs, and its body is the op's own
    // few vector instructions.  Consecutive instructions run in one loop, and
    // the step's terminal (a wait's yield, END, FORK) leaves it, with no
    // general pass -- whose per-lane decode, opcode-uniform lane match, class
    // branches, fold checks and epilogue cost ~2.4k cycles per instruction
    // (tools/stats_probe.py).  The semantics are the pass's,
    // instruction for instruction: the same counts n (the 2^22 cap), register
    // writes, node variable / binding / frame stores, hash terms and terminal
    // staging.  Anything else -- a rare op, a fused pair, a jump the lanes
    // take differently, an instruction that would fail (a bad node, frames
    // over the cap, an out-of-range target, the step cap) -- leaves the lanes
    // at its pc for the general pass, which executes it exactly as before.
    __device__ __forceinline__ void fast_run(Th& th, uint32_t slot, St& s) {
        const uint64_t rm = __builtin_amdgcn_ballot_w64(s.running);
        if (!rm) return;
        uint32_t fp = __builtin_amdgcn_readlane(s.pc, (uint32_t)__builtin_ctzll(rm));
        if (__builtin_amdgcn_ballot_w64(s.running && s.pc != fp)) return;  // lanes at different pcs
        const bool run = s.running;
        for (uint32_t k = 0; k < TW_FAST_MAX; ++k) {
            // (the image's last instruction goes to the general pass: running off
            // the end is its error, counted as it counts it)
            if (fp + 1u >= c.n_insns || __builtin_amdgcn_ballot_w64(run && s.n >= TW_STEP_CAP)) break;
            const uint2 in = P[fp];
            const uint32_t w = __builtin_amdgcn_readfirstlane(in.x);
            const int32_t imm = (int32_t)__builtin_amdgcn_readfirstlane(in.y);
            const uint32_t op = w & 0xFFu, a = (w >> 8) & 3u, b = w >> 16;
            uint32_t nx = fp + 1u;      // the next pc (uniform)
            uint32_t fin = T_NONE;      // a terminal: every running lane leaves the step
            if (op == TW_OP_FORK) {     // r[a] <- ref(child) at the terminal (TimedT.hs:326-342)
                const uint32_t node = b == 0xFFFFu ? th.w1 : (uint32_t)rg(th, b & 3u);
                if (__builtin_amdgcn_ballot_w64(run && node >= c.N)) break;
                csp(run, CW_CSP, csp_word((uint32_t)imm, a, 2u));  // the child's registers are the parent's
                csp(run, CW_CNODE, node);
                fin = T_SPAWN;
            } else if (op == TW_OP_WAIT_REL || op == TW_OP_WAIT_ABS || op == TW_OP_WAIT_REG) {
                int64_t wt;
                if (op == TW_OP_WAIT_REG) {
                    const int64_t ra = rg(th, a);
                    wt = now + (ra > 0 ? ra : 0);
                } else {
                    const int64_t kt = K[imm];
                    wt = op == TW_OP_WAIT_REL ? now + kt : (kt > now ? kt : now);
                }
                s.yt = run ? wt : s.yt;
                fin = T_YIELD;
            } else if (op == TW_OP_END) {
                fin = T_EXIT;
            } else if (op == TW_OP_JMP) {
                if ((uint32_t)imm >= c.n_insns) break;
                nx = (uint32_t)imm;
            } else if (op >= TW_OP_JEQ && op <= TW_OP_JNEI) {
                if ((uint32_t)imm >= c.n_insns) break;
                const int64_t ra = rg(th, a), rb = rg(th, b & 3u), bi = (int64_t)(int16_t)b;
                const bool tk = op == TW_OP_JEQ ? ra == rb : op == TW_OP_JNE ? ra != rb : op == TW_OP_JLT ? ra < rb
                              : op == TW_OP_JLE ? ra <= rb : op == TW_OP_JEQI ? ra == bi : ra != bi;
                const uint64_t tm = __builtin_amdgcn_ballot_w64(run && tk);
                if (tm != 0 && tm != rm) break;  // the lanes part ways: the general pass
                nx = tm ? (uint32_t)imm : nx;
            } else if (op == TW_OP_SETI || op == TW_OP_SETK || op == TW_OP_ADDI || op == TW_OP_MULI ||
                       op == TW_OP_MOV || op == TW_OP_ADD || op == TW_OP_SUB || op == TW_OP_NOW ||
                       op == TW_OP_NODE || op == TW_OP_MYTID) {
                const bool two = op == TW_OP_MOV || op == TW_OP_ADD || op == TW_OP_SUB;
                if (!two && op != TW_OP_MYTID && (b & TW_ALU_NSTORE)) break;  // a fused pair
                const int64_t ra = rg(th, a);
                const int64_t rb = two ? rg(th, b & 3u) : 0;
                int64_t v;
                if (op == TW_OP_SETI) v = imm;
                else if (op == TW_OP_SETK) v = K[imm];
                else if (op == TW_OP_ADDI) v = ra + (int64_t)imm;
                else if (op == TW_OP_MULI) v = ra * (int64_t)imm;
                else if (op == TW_OP_MOV) v = rb;
                else if (op == TW_OP_ADD) v = ra + rb;
                else if (op == TW_OP_SUB) v = ra - rb;
                else if (op == TW_OP_NOW) v = now;
                else if (op == TW_OP_NODE) v = (int64_t)th.w1;
                else v = (int64_t)(((uint64_t)th.w2 << 32) | slot);
                rs(th, a, run ? v : ra);
            } else if (op == TW_OP_NLOAD) {
                const int64_t x = gp(c.nvars)[nix(run ? th.w1 : 0u, b & 3u)];
                tw_vm_drain();
                if (run) rs(th, a, x);
            } else if (op == TW_OP_NSTORE) {
                const int64_t ra = rg(th, a);
                if (run) gp(c.nvars)[nix(th.w1, b & 3u)] = ra;
            } else if (op == TW_OP_TRACE) {
                if (c.trace_cap || (b & TW_TRACE_PAIR)) break;
                const int64_t ra = rg(th, a);
                hacc += run ? term(now, TW_KIND_TRACE | ((uint32_t)imm & 0xFFFFu), ra) : 0ull;
            } else if (op == TW_OP_CATCH) {
                const uint32_t nf = th_nfr(th);
                if (__builtin_amdgcn_ballot_w64(run && nf >= c.max_frames)) break;
                const uint32_t fv = (b << 16) | ((uint32_t)imm & 0xFFFFu);
                th.f0 = (run && nf == 0) ? fv : th.f0;
                th.f1 = (run && nf == 1) ? fv : th.f1;
                q1d = q1d || (run && nf < 2);
                if (run && nf >= 2) *fxp(slot, nf) = fv;  // deeper frames: the overflow area
                th.w0 = run ? (th.w0 & ~(15u << 16)) | ((nf + 1) << 16) : th.w0;
            } else if (op == TW_OP_LISTEN) {
                if ((uint32_t)imm >= c.n_sets) break;
                if (run) {
                    gp(c.bind)[bix(th.w1)] = (uint32_t)imm + 1;
                    gp(c.bind_own)[bix(th.w1)] = b ? th.w2 : 0xFFFFFFFFu;
                }
                th.w0 = (run && b) ? th.w0 | (F_OWNS << FL_SHIFT) : th.w0;
            } else if (op == TW_OP_UNLISTEN) {
                if (run) {
                    gp(c.bind)[bix(th.w1)] = 0;
                    gp(c.bind_own)[bix(th.w1)] = 0xFFFFFFFFu;
                }
            } else if (op != TW_OP_NOP) {
                break;  // a rare op: the general pass
            }
            STAT(K_INSN);
            s.n += run ? 1u : 0u;
            fp = nx;
            if (fin != T_NONE) {
                s.fin = run ? fin : s.fin;
                s.running = false;
                break;
            }
        }
        s.pc = run ? fp : s.pc;
    }

    // A fork whose child is the very next pop runs the child in place, in this
    // iteration (replica kernels).  TimedT's fork queues the child at now and
    // the parent at now + 1 (TimedT.hs:326-342); the child is PQ.minView's
    // next pick (TimedT.hs:242) when its queue key (now, key of the next
    // insertion counter value) is below every queued event's: under the
    // engine's (t, seq) order only if nothing else is queued at now, under
    // TW_TIE_LIFO always -- which is what pqueue's MinQueue does too, where an
    // insert whose key is <= the held minimum's becomes the new minimum.  For
    // those lanes the fork is carried out here exactly as the terminal and the
    // next pop would (TW_TIE_FORKFIRST: always the case, the child's key sorts
    // first): the child's thread id, slot and insertion counter value,
    // then the parent's queue entry at now + 1 and its record; the child's pop
    // is counted (event, clock, resume hash term on its node) and it becomes
    // the running thread, without its queue entry, the pop phase or a store
    // tail in between.  Returns true if some lane has a child to run.
    __device__ __forceinline__ bool fork_in_place(Th& th, uint32_t& slot, St& s) {
        const uint32_t kc = c.tie_mode == TW_TIE_FORKFIRST ? seq + 1u : c.tie_mode ? seq_key(c.tie_mode, seq + 1u)
                                                                                   : seq + 1u;
        bool ip = s.fin == T_SPAWN && status == TW_REP_RUNNING && d_ev < ev_room && seq + 1u < seq_top() &&
                  tidc != 0xFFFFFFFFu;
        if (!__builtin_amdgcn_ballot_w64(ip)) return false;
        if (far_dirty) far_min();
        bool has = near_n != 0;
        int64_t qt = nbase + (int64_t)(nrk >> 32);
        uint32_t qs = (uint32_t)nrk;
        const bool uf = fsrc >= 0 && (!has || tless(fmt, fms, qt, qs));
        qt = uf ? fmt : qt;
        qs = uf ? fms : qs;
        has = has || fsrc >= 0;
        ip = ip && (!has || tless(now, kc, qt, qs));
        if (!__builtin_amdgcn_ballot_w64(ip)) return false;
        if (ip) {
            STAT(K_SPAWN);
            const uint32_t csw = cg(CW_CSP), cdel = (csw >> 20) & 3u, cra = (csw >> 16) & 7u, cpc = csw & 0xFFFFu;
            int64_t ref;
            Th ch;
            uint32_t cslot = 0xFFFFFFFFu;
            bool ok;
            if (cdel & 2u) {
                ok = spawn(cpc, cg(CW_CNODE), rg(th, 0), rg(th, 1), rg(th, 2), rg(th, 3), ref, ch, cslot, false);
            } else {
                const uint4 a = qq[0], b = qq[WG];
                ok = spawn(cpc, cg(CW_CNODE), qa(a), qb(a), qa(b), qb(b), ref, ch, cslot, false);
            }
            if (ok) {
                // the parent: `wait (for 1 mcs)` (TimedT.hs:340) -- queued, record stored
                if (cra < 4) rs(th, cra, ref);
                th_set_pc(th, s.pc);
                enqueue(th, slot, now + 1);
                th.r0 = rg(th, 0); th.r1 = rg(th, 1); th.r2 = rg(th, 2); th.r3 = rg(th, 3);
                put_rec(slot, th);
                // the child's pop (TimedT.hs:241-247): counted, its resume term on its node
                STAT(K_POP);
                ++d_ev;
                final_t = now;
                if (ch.w1 != hnode) {
                    hash_flush();
                    hnode = ch.w1;
                }
                hacc += term0(now, TW_KIND_RESUME | th_pc(ch));
                th = ch;
                slot = cslot;
                rf[0] = ch.r0; rf[WG] = ch.r1; rf[2 * WG] = ch.r2; rf[3 * WG] = ch.r3;
                s.pc = th_pc(th);
                th.w0 |= F_STARTED << FL_SHIFT;
                s.running = s.pc < c.n_insns;
                pfail(!s.running, TW_REP_ERR_INSN);
                s.fin = s.running ? (uint32_t)T_NONE : (uint32_t)T_STOP;
                s.n = 0;
                s.yt = 0;
                if constexpr (FOLD) {
                    // a child that starts with a wait (`schedule`'s stub) yields
                    // here, without an interpreter pass for it
                    const bool w0 = s.running && ((PW[s.running ? s.pc : c.n_insns] >> 23) & 1u);
                    if (__builtin_amdgcn_ballot_w64(w0)) {
                        const uint2 wi = P[w0 ? s.pc : 0u];
                        const int64_t kt = K[w0 ? wi.y : 0u];
                        const int64_t w = (wi.x & 0xFFu) == TW_OP_WAIT_ABS ? (kt > now ? kt : now) : now + kt;
                        s.yt = w0 ? w : s.yt;
                        s.n = w0 ? 1u : s.n;
                        s.pc = w0 ? s.pc + 1u : s.pc;
                        s.fin = w0 ? (uint32_t)T_YIELD : s.fin;
                        s.running = s.running && !w0;
                    }
                }
            } else {
                s.fin = T_STOP;  // (a slot or counter failure: the terminal stores the parent)
            }
        }
        return true;
    }

    // Run the popped threads' continuations until each yields or ends (the
    // ContT continuation of TimedT.hs:343-355).  Called by every lane of the
    // wave (`run` = this lane popped a runnable thread), so the loop is
    // wave-uniform: each pass takes the pc of the first running lane, the
    // lanes at that pc ("me") execute its instruction with the opcode,
    // operands and immediate in scalar registers; register reads and writes
    // go to the lane's LDS register file, every other per-lane effect is a
    // select predicated on `me` (only the rare memory-effect ops open a
    // divergent region).  Lanes in lock-step take one pass per instruction.
    // Yield / fork / exit are recorded per lane and carried out after the
    // loop for all lanes at once.
    __device__ __forceinline__ void step(Th& th, uint32_t slot, bool run, uint32_t n0 = 0) {
        St s;
        uint32_t& pc = s.pc;
        uint32_t& fin = s.fin;
        int64_t& yt = s.yt;
        pc = th_pc(th);
        th.w0 = run ? th.w0 | (F_STARTED << FL_SHIFT) : th.w0;
        s.running = run && pc < c.n_insns;
        pfail(run && !s.running, TW_REP_ERR_INSN);
        fin = (run && !s.running) ? (uint32_t)T_STOP : (uint32_t)T_NONE;
        s.n = n0;  // (a JMP taken at the pop: jump_at_pop)
        yt = 0;
        STIME(ti0);
        for (;;) {
            const uint64_t mask = __builtin_amdgcn_ballot_w64(s.running);
            if (mask == 0) {
                // (replica kernels) a fork whose child is the very next pop: the
                // child runs in place, its lanes running again.  Not in the
                // sparse geometry, whose kernel would spill for it (there the
                // child takes its queue round trip: the same order either way)
                if constexpr (!LP && !PL && IP) {
                    STIME(tip0);
                    const bool more = fork_in_place(th, slot, s);
                    STIME(tip1);
                    STADD(K_CYC_IP, tip1 - tip0);
                    if (more) continue;
                }
                break;
            }
            if constexpr (FAST) {
                fast_run(th, slot, s);
                if (!__builtin_amdgcn_ballot_w64(s.running)) continue;
            }
            const uint32_t first = (uint32_t)__builtin_ctzll(__builtin_amdgcn_ballot_w64(s.running));
            // every lane fetches its own instruction; the pass runs the first running
            // lane's opcode in all lanes holding that opcode (their operands and
            // immediates stay per lane), so divergent lanes at different pcs still
            // share a pass when they execute the same kind of instruction
            const uint32_t lpc = pc < c.n_insns ? pc : c.n_insns;  // image padded by one NOP
            const uint2 in = P[lpc];
            const uint32_t lfl = PU[lpc];
            const uint32_t op = __builtin_amdgcn_readlane(in.x, first) & 0xFFu;
            const uint32_t fl = __builtin_amdgcn_readlane(lfl, first);
            // PL: a pass of a hot-class op (no U_FX) serves every running lane at any
            // hot-class op, each with its own uop fields; a rare op serves the
            // lanes holding that opcode
            const bool hot = !(fl & U_FX);
            // (opcode-uniform pass: the lanes holding the first lane's opcode and uop
            // flags -- a fused pair's flags depend on b, not only on the opcode)
            const bool at = PL ? (s.running & ((hot & !(lfl & U_FX)) | (!hot & ((in.x & 0xFFu) == op))))
                               : (s.running && (in.x & 0xFFu) == op && ((lfl ^ fl) & (FOLDJ ? ~U_FOLD : ~0u)) == 0);
            STAT(K_PASS);
            pass(th, slot, s, at, in.x, (int32_t)in.y, op, fl, lfl);
        }
        STIME(ti1);
        STADD(K_CYC_INTERP, ti1 - ti0);
        STIME(tt0);
        // ---- terminal actions (queue work only), then a fixed-shape store tail
        Th ch;
        ch.w0 = ch.w1 = ch.w2 = ch.w3 = ch.f0 = ch.f1 = ch.xl = ch.xh = 0;
        ch.r0 = ch.r1 = ch.r2 = ch.r3 = 0;
        uint32_t cslot = 0xFFFFFFFFu;
        if (run) th_set_pc(th, pc);
        // fork (TimedT.hs:326-342): the child is queued at now, then the parent waits 1 µs
        if (fin == T_SPAWN) {
            STAT(K_SPAWN);
            const uint32_t csw = cg(CW_CSP), cdel = (csw >> 20) & 3u, cra = (csw >> 16) & 7u, cpc = csw & 0xFFFFu;
            int64_t ref;
            bool ok;
            if (LP && c.lpb && (cdel & 2u) && cg(CW_CNODE) != th.w1) {
                // a fork onto another node (batched LP): a spawn record; the ref is
                // opaque (-1: refs name engine slots, and a cross-node throwTo is
                // outside LP mode anyway).  Not from a phase-1 node: the window's
                // phase 0 has finished by then.
                ok = !(c.phase && gp(c.phase)[th.w1]);
                if (ok) emit_spawn(now, cpc, lane_of(cg(CW_CNODE)), rg(th, 0), rg(th, 1), rg(th, 2), rg(th, 3));
                else fail(TW_REP_ERR_INSN);
                ref = -1;
            } else if (cdel & 2u) {
                ok = spawn(cpc, cg(CW_CNODE), rg(th, 0), rg(th, 1), rg(th, 2), rg(th, 3), ref, ch, cslot);
            } else {
                const uint4 a = qq[0], b = qq[WG];
                ok = spawn(cpc, cg(CW_CNODE), qa(a), qb(a), qa(b), qb(b), ref, ch, cslot);
            }
            if (!ok) {
                fin = T_STOP;
            } else {
                if (cra < 4) rs(th, cra, ref);
                if (LP && (cdel & 1u)) {
                    // the deliverer's resume pop (at now+1, on the sending node), then it ends
                    hash_add((uint32_t)rg(th, 2), term0(now + 1, TW_KIND_RESUME | (TW_PC_DELIVER_STUB + 2)));
                    ++d_ev;
                    final_t = now + 1 > final_t ? now + 1 : final_t;
                    fin = T_EXIT;
                } else {
                    yt = now + 1;
                    fin = T_YIELD;
                }
            }
        }
        STIME(tt0a);
        STADD(K_CYC_SPAWN, tt0a - tt0);
        if (fin == T_YIELD) enqueue(th, slot, yt);
        else if (fin == T_EXIT) die_prep(th, slot);
        STIME(tt0b);
        STADD(K_CYC_ENQ, tt0b - tt0a);
        run_commit();
        STIME(tt1);
        STADD(K_CYC_TERM, tt1 - tt0);
        store_tail(slot, th, fin == T_YIELD || fin == T_STOP, fin == T_EXIT, cslot, ch);
        if constexpr (LP) {
            // A child queued at now is usually the next pop (a deliverer's handler):
            // its record goes to the staging quads right away instead of the
            // prefetch's guess made before the step.  The store tail's 8 stores are
            // younger than that prefetch, so vmcnt(8) proves it has landed and
            // cannot overwrite these LDS writes.
            if (cslot != 0xFFFFFFFFu && near_n != 0 && nrs == cslot) {
                asm volatile("s_waitcnt vmcnt(8) ; tw:pf" ::: "memory");
                pfs[0] = make_uint4(ch.w0, ch.w1, ch.w2, ch.w3);
                pfs[WG] = make_uint4(ch.f0, ch.f1, ch.xl, ch.xh);
                pfs[2 * WG] = make_uint4((uint32_t)ch.r0, (uint32_t)((uint64_t)ch.r0 >> 32), (uint32_t)ch.r1,
                                         (uint32_t)((uint64_t)ch.r1 >> 32));
                pfs[3 * WG] = make_uint4((uint32_t)ch.r2, (uint32_t)((uint64_t)ch.r2 >> 32), (uint32_t)ch.r3,
                                         (uint32_t)((uint64_t)ch.r3 >> 32));
                pf_slot = cslot;
            }
        }
        STIME(tt2);
        STADD(K_CYC_STORE, tt2 - tt1);
    }
};

// ------------------------------------------------------------------ kernels
__global__ void __launch_bounds__(TW_WG) tw_init_kernel(Dev c, uint32_t main_pc, uint32_t main_node,
                                                       const int64_t* main_regs, const int64_t* nv_init,
                                                       const uint32_t* listen_init, int lp_mode, uint32_t seq0,
                                                       uint32_t tid0) {
    uint32_t r = blockIdx.x * TW_WG + threadIdx.x;
    // LP contexts keep a lane's scalar block and thread records contiguous
    // ([lane][SC_LP_STRIDE] words, 4 quads per slot): written one lane per
    // thread, every store of a wave would touch 64 lines (a batched C3 share
    // of 8,192 replicas has 33.6M lanes: 13 ms of a 97-ms step).  The
    // workgroup writes its 256 lanes' blocks and slot-0 records as one
    // contiguous span instead, word k*256 + t by thread t.
    if (lp_mode && c.sc_lp) {
        const size_t l0 = (size_t)blockIdx.x * TW_WG;
        uint64_t GAS* scb = gp(c.scal) + l0 * SC_LP_STRIDE;
        for (uint32_t k = 0; k < SC_LP_STRIDE; ++k) {
            const uint32_t w = k * TW_WG + threadIdx.x;
            const uint32_t f = w % SC_LP_STRIDE;
            const size_t l = l0 + w / SC_LP_STRIDE;
            if (l >= c.R || f >= SC_COUNT) continue;
            const bool hm = ((c.lp0 + (uint32_t)l) >> c.rep_lg) == main_node;
            uint64_t v = 0;
            v = (f == SC_THREADS || f == SC_PENDING_MAIN || f == SC_BUMP) ? (hm ? 1u : 0u) : v;
            v = f == SC_TIDC ? tid0 : v;  // main is tid 0 (TimedT.hs:272-280)
            v = f == SC_SEQ ? seq0 : v;
            v = f == SC_STATUS ? (uint64_t)TW_REP_RUNNING : v;
            scb[w] = v;
        }
        if (c.RQ == 1) {  // slot 0 (Lane::hrec): quad j of lane l at l * 4 + j (else below)
            uint4 GAS* pb = gp(c.slots) + l0 * 4;
            for (uint32_t k = 0; k < 4; ++k) {
                const uint32_t w = k * TW_WG + threadIdx.x;
                const uint32_t j = w & 3u;
                const size_t l = l0 + (w >> 2);
                if (l >= c.R) continue;
                const uint32_t gl = (c.lp0 + (uint32_t)l) >> c.rep_lg;
                const uint32_t rl = (c.lp0 + (uint32_t)l) & ((1u << c.rep_lg) - 1u);
                const bool hm = gl == main_node;
                uint4 q = make_uint4(0u, 0u, 0u, 0u);
                if (j == 0) q = make_uint4((main_pc & 0xFFFFu) | (F_MAIN << FL_SHIFT), main_node, hm ? 0u : 0xFFFFFFFFu, 0u);
                if (j >= 2 && main_regs && hm) {
                    const int64_t m0 = main_regs[(size_t)rl * 4 + (j - 2) * 2], m1 = main_regs[(size_t)rl * 4 + (j - 2) * 2 + 1];
                    q = make_uint4((uint32_t)m0, (uint32_t)((uint64_t)m0 >> 32), (uint32_t)m1, (uint32_t)((uint64_t)m1 >> 32));
                }
                pb[w] = q;
            }
        }
    }
    if (r >= c.R) return;
    // LP mode: lane r runs global node g (of replica rho, batched mode); only
    // the main node's lane holds the main thread
    const uint32_t g = lp_mode ? (c.lp0 + r) >> c.rep_lg : 0u;
    const uint32_t rho = lp_mode ? (c.lp0 + r) & ((1u << c.rep_lg) - 1u) : r;
    const bool has_main = !lp_mode || g == main_node;
    if (!(lp_mode && c.sc_lp && c.RQ == 1)) {  // (LP contexts: written above)
    for (uint32_t f = 0; f < SC_COUNT; ++f) gp(c.scal)[sc_ix(c, f, r)] = 0;
    gp(c.scal)[sc_ix(c, SC_THREADS, r)] = has_main ? 1 : 0;
    gp(c.scal)[sc_ix(c, SC_TIDC, r)] = tid0;  // main is tid 0 (TimedT.hs:272-280)
    gp(c.scal)[sc_ix(c, SC_SEQ, r)] = seq0;
    gp(c.scal)[sc_ix(c, SC_STATUS, r)] = TW_REP_RUNNING;
    gp(c.scal)[sc_ix(c, SC_PENDING_MAIN, r)] = has_main ? 1 : 0;
    gp(c.scal)[sc_ix(c, SC_BUMP, r)] = has_main ? 1 : 0;  // slot 0 = main
    uint4 GAS* p = gp(c.slots) + (c.RQ == 1 ? (size_t)r * 4 : (size_t)r);  // slot 0 (Lane::hrec)
    uint32_t w0 = (main_pc & 0xFFFFu) | (F_MAIN << FL_SHIFT);
    p[0] = make_uint4(w0, main_node, has_main ? 0u : 0xFFFFFFFFu, 0u);
    p[c.RQ] = make_uint4(0u, 0u, 0u, 0u);
    int64_t m[4] = {0, 0, 0, 0};
    if (main_regs && has_main)
        for (int i = 0; i < 4; ++i) m[i] = main_regs[(size_t)rho * 4 + i];
    p[2 * c.RQ] = make_uint4((uint32_t)m[0], (uint32_t)((uint64_t)m[0] >> 32), (uint32_t)m[1], (uint32_t)((uint64_t)m[1] >> 32));
    p[3 * c.RQ] = make_uint4((uint32_t)m[2], (uint32_t)((uint64_t)m[2] >> 32), (uint32_t)m[3], (uint32_t)((uint64_t)m[3] >> 32));
    }
    if (lp_mode) {
        if (nv_init)
            for (uint32_t i = 0; i < 4; ++i) gp(c.nvars)[(size_t)i * c.R + r] = nv_init[(size_t)g * 4 + i];
        gp(c.bind_own)[r] = 0xFFFFFFFFu;
        gp(c.bind_rel)[r] = 0xFFFFFFFEu;
        if (listen_init) gp(c.bind)[r] = listen_init[g];
        gp(c.inbox_n)[r] = 0;
        gp(c.inbox_n)[c.R + r] = 0;
        if (c.lpb) gp(c.spawn_n)[r] = 0;
        gp(c.wake)[r] = INT64_MAX;
        lp_mark(c, r, 0);  // marked for the first window: it serves every node
        if (c.rw && (((r >> c.rep_lg) & ((1u << TW_CHUNK_LG) - 1u)) == 0)) gp(c.cw_min)[cw_idx(c, r)] = INT64_MAX;
        if ((r & ((1u << TW_SUB_LG) - 1u)) == 0) {
            gp(c.sb_scan)[r >> TW_SUB_LG] = 0xFFFFFFFFu;
            gp(c.sb_min)[r >> TW_SUB_LG] = INT64_MAX;
        }
        return;
    }
    if (nv_init)
        for (uint32_t i = 0; i < c.N * 4; ++i) gp(c.nvars)[(size_t)i * c.R + r] = nv_init[i];
    for (uint32_t n = 0; n < c.N; ++n) {
        gp(c.bind_own)[(size_t)n * c.R + r] = 0xFFFFFFFFu;
        gp(c.bind_rel)[(size_t)n * c.R + r] = 0xFFFFFFFEu;
    }
    if (listen_init)
        for (uint32_t n = 0; n < c.N; ++n) gp(c.bind)[(size_t)n * c.R + r] = listen_init[n];
}

// LDS per workgroup: near heap keys + slots, the running threads' register
// files, the cold words, then the program image and constant pool, so
// instruction fetch and time constants never leave the CU.
template <int WG, int NC, bool LP = false, bool RUNS = true>
__host__ __device__ constexpr size_t fixed_lds_bytes() {
    return (size_t)(LP || !RUNS ? 4 : 5) * WG * 16 + (size_t)(LP || !RUNS ? 0 : RQ_COUNT) * WG * 16 + (size_t)NC * WG * 12 +
           (size_t)4 * WG * 8 + (size_t)2 * WG * 16 + (size_t)(cw_count<LP>() + (LP ? DW_COUNT : 0)) * WG * 4;
}

// WG replicas per workgroup share its LDS; TPW of each wave's 64 lanes carry a
// replica (64, or TW_HALF_LANES for the half geometry: twice the waves).
// RUNS = false (the compact geometry): no far runs, and built for two waves
// per SIMD (<= 256 registers, half the LDS of a dense lane), so 1M-replica
// batches keep two workgroups per CU
// LP lanes' prologue: the near spill's entries and the far heap's top loaded
// together (round 6: C5 1,366 -> 1,341 ms, C4 flat; TW_LP_PRO=0 for the A/B)
#ifndef TW_LP_PRO
#define TW_LP_PRO 1
#endif
template <bool LP, int WG, int NC, int TPW = 64, bool RUNS = true, bool GS = false, bool PRW = false, bool IP = false>
__global__ void __launch_bounds__(WG * 64 / TPW)
    __attribute__((amdgpu_waves_per_eu(LP ? TW_LP_WAVES : !RUNS ? 2 : (WG * 64 / TPW + 255) / 256,
                                       LP ? TW_LP_WAVES : 2)))
tw_run_kernel(Dev c, int64_t t_end, uint64_t max_events, uint32_t budget) {
    constexpr bool HR = !LP && RUNS;
    // device-driven windows: the window, its work list and whether this is the
    // window's first tick (the only one that drains inboxes) come from the device
    bool fresh = true;
    uint32_t ph = 0;
    int64_t lwin = 0;  // the lookahead (per-replica windows: t_end is the lane's replica's)
    // LP: the window's work list (workgroups past it leave before staging the program)
    static_assert(TW_LP_NB == 1, "the LP grid serves one work-list bucket");
    uint32_t lp_n = 0;
    if (LP && c.win) {
        // (both lists' lengths load with the window words: a workgroup past the
        // list -- most of a light tick's grid -- leaves after one round trip)
        const uint32_t n0 = gp(c.act_n)[0], n1 = gp(c.act_n)[TW_LP_NB];
        const int64_t GAS* w = gp(c.win);
        const int64_t fl = w[WN_FLAGS];
        lwin = w[WN_L];
        t_end = w[WN_T] + w[WN_L] - 1;
        c.act_cur = (uint32_t)w[WN_ACT];
        c.wid = (uint32_t)w[WN_WID];
        ph = (uint32_t)w[WN_PHASE];
        if (fl & WN_DONE) return;
        fresh = (fl & (ph ? WN_PH1FRESH : WN_FRESH)) != 0;
        lp_n = c.act_cur ? n1 : n0;
        if ((size_t)blockIdx.x * WG >= lp_n) return;
    } else if (LP) {
        lp_n = gp(c.act_n)[c.act_cur * TW_LP_NB];
        if ((size_t)blockIdx.x * WG >= lp_n) return;
    }
    extern __shared__ __attribute__((aligned(16))) uint64_t lds_raw[];
    uint4 LAS* s_pf = (uint4 LAS*)lds_raw;
    uint4 LAS* s_rq = s_pf + (HR ? 5 : 4) * WG;  // (staging quad 4 holds a far run's next entry: runs only)
    uint64_t LAS* s_k = (uint64_t LAS*)(s_rq + (HR ? RQ_COUNT : 0) * WG);
    int64_t LAS* s_rf = (int64_t LAS*)(s_k + NC * WG);
    uint4 LAS* s_q = (uint4 LAS*)((uint8_t LAS*)s_pf + qq_lds_offset<WG, NC, HR>());  // (= s_rf + 4 * WG)
    uint32_t LAS* s_s = (uint32_t LAS*)(s_q + 2 * WG);
    uint32_t LAS* s_cw = s_s + NC * WG;
    uint2 LAS* s_p = (uint2 LAS*)(s_cw + (cw_count<LP>() + (LP ? DW_COUNT : 0)) * WG);
    int64_t LAS* s_c = (int64_t LAS*)(s_p + c.n_insns + 1);
    uint32_t LAS* s_u = (uint32_t LAS*)(s_c + c.n_consts);
    uint32_t LAS* s_l = s_u + c.n_insns + 1;
    uint32_t LAS* s_w = s_l + c.n_sets * c.n_kinds;  // pop words [n_insns + 1]
    {
        for (uint32_t i = threadIdx.x; i <= c.n_insns; i += WG * 64 / TPW) {
            const uint2 in = gp(c.insns)[i];
            s_p[i] = in;
            uint32_t u = uop_insn(in.x);
            auto is_end = [&](uint32_t j) { return j < c.n_insns && (gp(c.insns)[j].x & 0xFFu) == TW_OP_END; };
            if (LP && TW_LP_FOLDJ && i < c.n_insns) {  // (Lane::FOLDJ: a jump only)
                const uint32_t nop = i + 1u < c.n_insns ? gp(c.insns)[i + 1u].x & 0xFFu : TW_OP_NOP;
                u |= U_JM(uop_of(nop)) != JM_NONE ? U_NJ : 0u;
            }
            if (LP && TW_LP_FORKN && c.lpb && i + 2u < c.n_insns && (in.x & 0xFFu) == TW_OP_FORK &&
                (in.x >> 16) != 0xFFFFu) {  // (Lane::fork_loop)
                const uint32_t w1 = gp(c.insns)[i + 1u].x;
                const uint2 j2 = gp(c.insns)[i + 2u];
                const uint32_t op2 = j2.x & 0xFFu;
                u |= ((w1 & 0xFFu) == TW_OP_ADDI && !((w1 >> 16) & TW_ALU_NSTORE) && op2 >= TW_OP_JEQ &&
                      op2 <= TW_OP_JNEI && j2.y == i) ? U_FL : 0u;
            }
            if (HR && i < c.n_insns) {  // (Lane::FOLD)
                u |= is_end(i + 1u) ? U_NE : 0u;
                u |= is_end(i + 2u) ? U_NE2 : 0u;
                u |= (U_JM(u) != JM_NONE && is_end((uint32_t)in.y)) ? U_JE : 0u;
                const uint32_t nop = i + 1u < c.n_insns ? gp(c.insns)[i + 1u].x & 0xFFu : TW_OP_NOP;
                u |= (nop == TW_OP_WAIT_REL || nop == TW_OP_WAIT_ABS) ? U_NW : 0u;
                u |= U_JM(uop_of(nop)) != JM_NONE ? U_NJ : 0u;
            }
            s_u[i] = u;
        }
        for (uint32_t i = threadIdx.x; i < c.n_consts; i += WG * 64 / TPW) s_c[i] = gp(c.consts)[i];
        for (uint32_t i = threadIdx.x; i < c.n_sets * c.n_kinds; i += WG * 64 / TPW) s_l[i] = gp(c.lpc)[i];
        // pop_word(pc): the pc a resumed thread starts at (an unconditional JMP's
        // target; bit 16 = the JMP was taken), and whether that pc / the next are
        // THROW_TOs (bits 17, 18) with their victim registers (bits 19-20, 21-22);
        // bit 23: the instruction at pc itself is a wait (fork_in_place)
        for (uint32_t i = threadIdx.x; i <= c.n_insns; i += WG * 64 / TPW) {
            uint32_t w = i;
            if (i < c.n_insns) {
                const uint2 in = gp(c.insns)[i];
                const bool j = (in.x & 0xFFu) == TW_OP_JMP && (uint32_t)in.y < c.n_insns;
                const uint32_t t = j ? (uint32_t)in.y : i;
                const uint32_t w0 = gp(c.insns)[t].x, w1 = gp(c.insns)[t + 1u].x;  // (padded by one NOP)
                const uint32_t op = in.x & 0xFFu;
                w = t | (j ? 1u << 16 : 0u) | ((w0 & 0xFFu) == TW_OP_THROW_TO ? 1u << 17 : 0u) |
                    ((w1 & 0xFFu) == TW_OP_THROW_TO ? 1u << 18 : 0u) | (((w0 >> 8) & 3u) << 19) |
                    (((w1 >> 8) & 3u) << 21) | ((op == TW_OP_WAIT_REL || op == TW_OP_WAIT_ABS) ? 1u << 23 : 0u);
            }
            s_w[i] = w;
        }
        __syncthreads();
    }
    if (TPW < 64 && (threadIdx.x & 63u) >= TPW) return;
    const uint32_t wbase = (threadIdx.x >> 6) * TPW;  // the wave's first lane in the LDS layout
    const uint32_t li = wbase + (threadIdx.x & 63u);
    // GS (LP contexts of more than TW_LP_GRID workgroups of lanes): the
    // workgroups walk the window's work list grid-stride, so a list of a few
    // thousand lanes out of millions dispatches no empty workgroups (the loop
    // costs registers: the smaller LP contexts launch one workgroup per WG lanes)
    for (uint32_t blk = blockIdx.x;; blk += gridDim.x) {
        do {
            uint32_t r = blk * WG + li;
            if (LP) {
                const uint32_t i = blk * WG + li;
                if (i >= lp_n) break;  // (the next block of the work list)
                r = gp(c.act)[(size_t)c.act_cur * TW_LP_NB * c.R + i];
            }
            if (r >= c.R) break;  // (the next block of the work list)
            STIME(tpro0);
            if (LP && c.phase && gp(c.phase)[(c.lp0 + r) >> c.rep_lg] != ph) break;  // the other phase's node
            // the lane's scalar block: [field][replica] for replicas (a wave's
            // lanes move in lock-step: one coalesced line per field), a
            // contiguous [lane][SC_LP_STRIDE] block for LP lanes (work lists
            // are sparse: one or two lines per lane instead of one per field)
            uint64_t* sc = gp(c.scal) + (LP ? (size_t)r * SC_LP_STRIDE : (size_t)r);
            const size_t SR = LP ? 1 : c.R;
            const size_t R = c.R;
            if (sc[SC_STATUS * SR] != TW_REP_RUNNING) break;  // (the next block of the work list)
            // this lane's window end (PRW: per-replica windows, Dev::rw -- a per-lane value)
            const int64_t te = (LP && PRW) ? rw_tend(c, r, lwin) : t_end;
            // LP: a node with no live thread, nothing to drain, no due run and no
            // spawn record has nothing to do in this window (every live thread holds
            // its one queued event; a superseded entry left behind pops without effect
            // whenever the node wakes again).  A light inbox (<= TW_LIGHT records) is
            // drained into the queue at the window's first tick; a heavy one was
            // sorted by tw_lp_due into this window's due run and the records due later.
            uint32_t n_in = 0, ipar = 0;
            bool ilight = false;
            if (LP) {
                ilight = ib_cap(c, r) <= TW_LIGHT;
                ipar = (c.dpar && c.win && ilight) ? (c.wid & 1u) : 0u;  // the buffer the last window filled
                n_in = gp(c.inbox_n)[(size_t)ipar * R + r];
                const bool drain = fresh && n_in != 0 && ilight;
                if (sc[SC_LIVE * SR] == 0 && sc[SC_PENDING_MAIN * SR] == 0 && !drain && sc[SC_DUE_H * SR] >= sc[SC_DUE_N * SR] &&
                    !(c.lpb && gp(c.spawn_n)[r]))
                    break;  // (the next block of the work list)
            }

            Lane<LP, WG, NC, RUNS, IP> L;
            L.c = c;
            L.r = r;
            L.nk = s_k + li;
            L.ns = s_s + li;
            L.rf = s_rf + li;
            L.qq = s_q + li;
            L.cw = s_cw + li;
            L.pfs = s_pf + li;
            L.rq = s_rq + li;
            L.pfs_wave = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(s_pf + wbase));
            L.P = s_p;
            L.PU = s_u;
            L.PW = s_w;
            L.K = s_c;
            L.LPC = s_l;
            L.pf_slot = 0xFFFFFFFFu;
            L.prun = -1;
            L.hacc = 0;
            L.hnode = 0xFFFFFFFFu;
            L.now = (int64_t)sc[SC_NOW * SR]; L.final_t = (int64_t)sc[SC_FINAL_T * SR];
            L.seq = (uint32_t)sc[SC_SEQ * SR]; L.tidc = (uint32_t)sc[SC_TIDC * SR]; L.live = (uint32_t)sc[SC_LIVE * SR];
            const uint32_t near_n0 = (uint32_t)sc[SC_NEAR_N * SR];
            L.far_n = (uint32_t)sc[SC_FAR_N * SR];
            L.status = (uint32_t)sc[SC_STATUS * SR];
            L.free_n = (uint32_t)sc[SC_FREE_N * SR]; L.ftop = (uint32_t)sc[SC_FTOP * SR]; L.bump = (uint32_t)sc[SC_BUMP * SR];
        #pragma unroll
            for (int w = 0; w < cw_count<LP>(); ++w) L.cs(w, 0);
            L.cs(CW_MAINEXC, (uint32_t)sc[SC_MAIN_EXC * SR]);
            L.cs(CW_TMO, (uint32_t)sc[SC_TMO_CTR * SR]);
            if constexpr (!LP) L.cs(CW_TRN, (uint32_t)sc[SC_TRACE_N * SR]);
            const uint64_t events0 = sc[SC_EVENTS * SR];
            const uint64_t ev_room64 = max_events > events0 ? max_events - events0 : 0;
            const uint32_t ev_room = ev_room64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)ev_room64;
            L.t_end = te;
            L.ev_room = ev_room;
            L.d_ev = 0;
            L.d_th = 0;
            if constexpr (LP && TW_LP_PRO) {
                // (loaded whether or not the heap holds anything, so the load
                // goes out with the scalar block's instead of after it; CW_FT*
                // are read only while far_n > 0)
                L.set_ftop(c.Q ? L.far_ld(0) : make_uint4(0u, 0u, 0u, 0u));
            } else {
                if (L.far_n) L.set_ftop(L.far_ld(0));
            }
            L.rlc_link = 0xFFFFFFFFu;
            L.rlc_rev = 0;
            L.oo = 0;
            if constexpr (LP) {
                L.oo = gp(c.out_off)[(c.lp0 + r) >> c.rep_lg];  // (the lane's node: every thread of an LP lane runs on it)
                const uint32_t dn = (uint32_t)sc[SC_DUE_N * SR], dh = (uint32_t)sc[SC_DUE_H * SR];
                const size_t ib = ib_base(c, r);
                L.ds(DW_IB, (uint32_t)ib);
                L.ds(DW_HN, dh | (dn << 16));
                L.ds(DW_SQ0, (uint32_t)sc[SC_DUE_SEQ * SR]);
                uint4 h = make_uint4(0, 0, 0, 0);
                if (dh < dn) h = gp(c.due)[(ib + (size_t)dh * ib_stride(c, !ilight)) * 2];
                L.ds(DW_TL, h.x);
                L.ds(DW_TH, h.y);
                L.ds(DW_BSET, gp(c.bind)[r]);  // (LP: bix(node) = the lane itself)
                L.ds(DW_BOWN, gp(c.bind_own)[r]);
                L.ds(DW_BREL, gp(c.bind_rel)[r]);
            }
            if constexpr (HR) {
                uint32_t rh4[TW_RUNS];
        #pragma unroll
                for (int j = 0; j < TW_RUNS; ++j) {
                    // (no far runs configured, e.g. LP nodes: nothing to load)
                    const uint32_t rh = c.Cr ? (uint32_t)sc[(SC_RH0 + j) * SR] : 0u;
                    const uint32_t rn = c.Cr ? (uint32_t)sc[(SC_RC0 + j) * SR] : 0u;
                    rh4[j] = rh;
                    uint4 h = make_uint4(0, 0, 0, 0), s2 = h, u = h;
                    if (rn) {
                        h = *L.run_at(j, rh);
                        uint32_t tp = rh + rn - 1;
                        if (tp >= c.Cr) tp -= c.Cr;
                        u = *L.run_at(j, tp);
                        if (rn >= 2) s2 = *L.run_at(j, rh + 1 == c.Cr ? 0 : rh + 1);
                    }
                    *L.rqp(RQ_HEAD + j) = h;
                    *L.rqp(RQ_SEC + j) = s2;
                    *L.rqp(RQ_TAIL + j) = make_uint4(u.x, u.y, u.w, rn);
                }
                *L.rqp(RQ_IDX) = make_uint4(rh4[0], rh4[1], rh4[2], rh4[3]);
            }
            L.far_min();
            // near heap: the spill area holds heap positions [0, near_n) verbatim with
            // absolute times; re-keyed to this launch's base (a common shift keeps the
            // heap order) they go back in place, without sifting.  An entry too far
            // ahead for a 32-bit key (or an oversized spill) takes the pushing path.
            L.nbase = L.now;
            L.near_init();
            if constexpr (LP && TW_LP_PRO) {
                // (an LP lane reloads its spill every window: its entries are
                // loaded together, one round trip, instead of one after another)
                uint4 se[NC];
                bool fits = near_n0 <= (uint32_t)NC;
        #pragma unroll
                for (uint32_t j = 0; j < (uint32_t)NC; ++j)
                    se[j] = (fits && j < near_n0) ? gp(c.near_spill)[(size_t)j * R + r] : make_uint4(0u, 0u, 0u, 0u);
        #pragma unroll
                for (uint32_t j = 0; j < (uint32_t)NC; ++j)
                    fits = fits && (j >= near_n0 || (uint64_t)(ent_t(se[j]) - L.nbase) < 0xFFFFFFFFull);
                if (fits) {
        #pragma unroll
                    for (uint32_t j = 0; j < (uint32_t)NC; ++j) {
                        if (j < near_n0) {
                            L.nk[j * WG] = L.nkey(ent_t(se[j]), se[j].w);
                            L.ns[j * WG] = se[j].z;
                        }
                    }
                    L.near_n = near_n0;
                    L.nrk = near_n0 ? L.nkey(ent_t(se[0]), se[0].w) : ~0ull;
                    L.nrs = near_n0 ? se[0].z : 0u;
                } else {
                    for (uint32_t j = 0; j < near_n0; ++j) {
                        uint4 e = gp(c.near_spill)[(size_t)j * R + r];
                        if (L.near_n < NC && (uint64_t)(ent_t(e) - L.nbase) < 0xFFFFFFFFull) {
                            L.near_push(ent_t(e), e.w, e.z);
                            continue;
                        }
                        L.push_far(ent_t(e), e.w, e.z);
                    }
                }
            } else {
                bool fits = near_n0 <= (uint32_t)NC;
                for (uint32_t j = 0; j < near_n0 && fits; ++j)
                    fits = (uint64_t)(ent_t(gp(c.near_spill)[(size_t)j * R + r]) - L.nbase) < 0xFFFFFFFFull;
                if (fits) {
                    for (uint32_t j = 0; j < near_n0; ++j) {
                        const uint4 e = gp(c.near_spill)[(size_t)j * R + r];
                        L.nk[j * WG] = L.nkey(ent_t(e), e.w);
                        L.ns[j * WG] = e.z;
                    }
                    L.near_n = near_n0;
                    L.nrk = L.nk[0];
                    L.nrs = L.ns[0];
                } else {
                    for (uint32_t j = 0; j < near_n0; ++j) {
                        uint4 e = gp(c.near_spill)[(size_t)j * R + r];
                        if (L.near_n < NC && (uint64_t)(ent_t(e) - L.nbase) < 0xFFFFFFFFull) {
                            L.near_push(ent_t(e), e.w, e.z);
                            continue;
                        }
                        L.push_far(ent_t(e), e.w, e.z);  // the thread's F_NEARQ hint only speeds up throwTo
                    }
                }
            }

            if (LP && fresh && n_in != 0 && ilight) {
                // delivery records addressed to this node become phantom deliverer
                // threads, inserted in (t, link, payload, src, kind) order (rec_less, the
                // order tw_lp_due gives a heavy lane's due run) so queue seqs are
                // deterministic whatever order the records arrived in
                const size_t ib = (size_t)ipar * c.ib_total + ib_base(c, r), ist = ib_stride(c, false);
                const uint32_t cap = ib_cap(c, r);  // (an overflowed inbox -- lp_err set -- keeps its first cap)
                if (n_in > cap) {
                    L.fail(TW_REP_ERR_QUEUE);
                    n_in = cap;
                }
                uint32_t used = 0;  // bitmask, n_in <= TW_LIGHT = 32
                for (uint32_t k = 0; k < n_in && L.status == TW_REP_RUNNING; ++k) {
                    int best = -1;
                    uint4 ba = make_uint4(0, 0, 0, 0), bb = ba;
                    for (uint32_t j = 0; j < n_in; ++j) {
                        if (used & (1u << j)) continue;
                        const uint4 GAS* q = gp(c.inbox) + (ib + (size_t)j * ist) * 2;
                        uint4 ea = q[0], eb = q[1];
                        if (best < 0 || rec_less(ea, eb, ba, bb)) { best = (int)j; ba = ea; bb = eb; }
                    }
                    used |= 1u << best;
                    int64_t ta = ent_t(ba);
                    if (ta < L.now) {  // delivered after the node ran past it: not conservative
                        L.fail(TW_REP_ERR_INSN);
                        break;
                    }
                    uint32_t s = L.alloc_slot();
                    if (s == 0xFFFFFFFFu) break;
                    Th ph;
                    ph.w0 = ((TW_PC_DELIVER_STUB + 1) & 0xFFFFu) | ((F_STARTED | F_PHANTOM) << FL_SHIFT);
                    ph.w1 = (c.lp0 + r) >> c.rep_lg;
                    ph.w2 = 0xFFFFFFFEu;  // never a throwTo target
                    ph.w3 = 0;
                    ph.f0 = ph.f1 = ph.xl = ph.xh = 0;
                    ph.r0 = (int64_t)(((uint64_t)ba.w << 32) | ba.z);  // payload
                    ph.r1 = bb.x;                                     // link
                    ph.r2 = bb.z;                                     // sending node
                    ph.r3 = bb.y;                                     // kind
                    L.enqueue(ph, s, ta);
                    L.put_rec(s, ph);
                }
                gp(c.inbox_n)[(size_t)ipar * R + r] = 0;
            }
            if (LP && c.lpb) {
                // batched LP: children forked onto this node by another node of the
                // replica (emit_spawn), queued at their fork time
                uint32_t nsp = gp(c.spawn_n)[r];
                if (nsp) {
                    if (nsp > TW_SPN) {
                        L.fail(TW_REP_ERR_QUEUE);
                        nsp = TW_SPN;
                    }
                    for (uint32_t k = 0; k < nsp && L.status == TW_REP_RUNNING; ++k) {
                        const uint4 GAS* q = gp(c.spawn) + ((size_t)k * R + r) * 4;
                        const uint4 a = q[0], b = q[1], d = q[2], e = q[3];
                        const int64_t t = ent_t(a);
                        if (t < L.now) {  // the lane already ran past the fork time: not conservative
                            L.fail(TW_REP_ERR_INSN);
                            break;
                        }
                        const uint32_t s = L.alloc_slot();
                        if (s == 0xFFFFFFFFu) break;
                        if (L.tidc == 0xFFFFFFFFu) {
                            L.fail(TW_REP_ERR_COUNTER);
                            break;
                        }
                        Th ch;
                        ch.w0 = b.x & 0xFFFFu;
                        ch.w1 = (c.lp0 + r) >> c.rep_lg;
                        ch.w2 = L.tidc++;
                        ch.w3 = 0;
                        ch.f0 = ch.f1 = ch.xl = ch.xh = 0;
                        ch.r0 = (int64_t)(((uint64_t)a.w << 32) | a.z);
                        ch.r1 = (int64_t)(((uint64_t)d.y << 32) | d.x);
                        ch.r2 = (int64_t)(((uint64_t)d.w << 32) | d.z);
                        ch.r3 = (int64_t)(((uint64_t)e.z << 32) | e.x);
                        ++L.d_th;
                        L.enqueue(ch, s, t);
                        L.put_rec(s, ch);
                    }
                    gp(c.spawn_n)[r] = 0;
                }
            }

        #ifdef TW_STATS
            for (int i = 0; i < P_COUNT; ++i) L.st[i] = 0;
            {
                STIME(tpro1);
                STADDL(K_CYC_PRO, tpro1 - tpro0);
            }
        #endif
            uint32_t pending_main = (uint32_t)sc[SC_PENDING_MAIN * SR];
            // nothing loaded before the loop may stay pending into it (a loop-header
            // wait would otherwise drain the counter on every iteration)
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
            // The loop is wave-uniform: a lane that stops (quiescence, t_end, event
            // cap, error) just idles through the remaining iterations, so no per-lane
            // break/continue splits the wave's control flow.
            bool alive = L.status == TW_REP_RUNNING;
            for (uint32_t it = 0; it < budget; ++it) {
                if (!__builtin_amdgcn_ballot_w64(alive)) break;
                STIME(tl0);
                STATL(K_ITER);  // lane-iterations, idle lanes included (pops / this = lane efficiency)
                Th th;
                uint32_t slot = 0;
                bool run = false;
                // the rare cases (main's first run, quiescence, the event cap) behind one
                // wave-uniform branch; the common path is a single divergent region
                const bool rare = alive && (pending_main || L.live == 0 || L.d_ev >= ev_room);
                if (__builtin_amdgcn_ballot_w64(rare)) {
                    if (rare && pending_main) {  // runInSandbox main (TimedT.hs:237): runs at t=0, not a pop
                        pending_main = 0;
                        L.pf_slot = 0xFFFFFFFFu;
                        L.fetch_rec(0, th);
                        L.rf[0] = th.r0; L.rf[WG] = th.r1; L.rf[2 * WG] = th.r2; L.rf[3 * WG] = th.r3;
                        L.hnode = th.w1;
                        run = true;
                    } else if (rare) {  // whileM_ notDone, or this launch's event cap
                        if (!LP && L.live == 0) L.status = TW_REP_DONE;  // an LP may still receive records
                        alive = false;
                    }
                }
                bool popping = alive && !rare;
                L.q1d = false;
                {
                    // PQ.minView: the min of the near root and the far sources
                    if (L.far_dirty) L.far_min();
                    const bool use_near = L.near_n != 0;
                    const int64_t tn = L.nbase + (int64_t)(L.nrk >> 32);
                    const bool use_far = L.fsrc >= 0 && (!use_near || tless(L.fmt, L.fms, tn, (uint32_t)L.nrk));
                    const int64_t t = use_far ? L.fmt : tn;
                    const uint32_t sq = use_far ? L.fms : (uint32_t)L.nrk;
                    slot = use_far ? L.fmsl : (use_near ? L.nrs : 0u);
                    STIME(ts1);
                    STADDL(K_CYC_SEL, ts1 - tl0);
                    // parked beyond t_end (an empty queue cannot happen while live > 0)
                    const bool parked = popping && ((!use_near && !use_far) || t > te);
                    alive = parked ? false : alive;
                    popping = popping && !parked;
                    if (popping) {
                        {
                            const bool due = LP && use_far && L.fsrc == 0;
                            if (due) L.due_pop(th, slot, sq);
                            else L.fetch_rec(slot, th);  // prefetched copy or HBM
                            STIME(ts2);
                            STADDL(K_CYC_FETCH, due ? 0 : ts2 - ts1);
                            STADDL(K_CYC_DUE, due ? ts2 - ts1 : 0);
                            if (due) {
                            } else if (!use_far) L.near_pop();
                            else if (L.fsrc == TW_RUNS) {
                                // (drained: the heap walk issues loads whose values go
                                // unused; left in flight, they made the compiler wait
                                // vmcnt(0) -- for the record prefetch and the last
                                // pass's stores -- at the top of every interpreter
                                // pass of every step, tools/waitcnt_audit.py)
                                L.far_pop();
                                tw_vm_drain();
                            } else L.run_pop(L.fsrc);
                            STIME(ts3);
                            STADDL(K_CYC_QPOP, ts3 - ts2);
                            if (slot == L.pf_slot) L.pf_slot = 0xFFFFFFFFu;
                            if (th.w3 != sq) {
                                STATL(K_SUPERSEDED);  // superseded by a throwTo re-stamp
                            } else {
                                STATL(K_POP);
                                // curTime .= timestamp (TimedT.hs:241-247)
                                th.w3 = 0;
                                --L.live;
                                L.now = t;
                                if (t - L.nbase > (int64_t)0x7FFFFFFF) L.near_rebase(t);
                                L.hnode = th.w1;
                                L.rf[0] = th.r0; L.rf[WG] = th.r1; L.rf[2 * WG] = th.r2; L.rf[3 * WG] = th.r3;
                                // LP phantom = the deliverer's wake, already counted and hashed by the sender
                                const bool phantom = LP && (th_flags(th) & F_PHANTOM);
                                if (!phantom) {
                                    L.final_t = LP ? (t > L.final_t ? t : L.final_t) : t;
                                    ++L.d_ev;
                                }
                                const uint32_t exc = th_exc(th);  // asyncExceptions . at tid <<.= Nothing (:252)
                                if (exc) {
                                    const int64_t val = th_xval(th);
                                    th_set_exc(th, 0);
                                    th.xl = th.xh = 0;
                                    L.q1d = true;
                                    L.hacc += term0(t, TW_KIND_EXC | exc);
                                    if (!(th_flags(th) & (F_STARTED | F_MAIN))) {  // escapes launchTimedT (:252-263)
                                        L.status = TW_REP_ABORTED;
                                        L.cs(CW_MAINEXC, exc);
                                        L.put_rec(slot, th);
                                    } else {
                                        run = L.unwind(th, slot, exc, val);
                                    }
                                } else {
                                    if (!phantom) L.hacc += term0(t, TW_KIND_RESUME | th_pc(th));
                                    run = true;
                                }
                            }
                        }
                    }
                }
                if (!popping) slot = 0u;  // main's first run is slot 0; idle lanes do not use it
                // (the compact geometry: neither -- C2's threads resume at no JMP
                // and throw nothing, and its per-pop cost is the bound)
                uint32_t pw = 0, n0 = 0;
                if constexpr (RUNS) n0 = L.jump_at_pop(th, run, pw);
                if constexpr (HR) L.stage_victims(slot, run, n0, pw);
                STIME(tp0);
                L.prefetch_all(run ? slot : 0xFFFFFFFFu);
                STIME(tl1);
                STADDL(K_CYC_PF, tl1 - tp0);
                STADDL(K_CYC_POP, tl1 - tl0);
                L.step(th, slot, run, n0);
                STIME(th0);
                L.hash_flush_all();
                STIME(th1);
                STADDL(K_CYC_HASH, th1 - th0);
                alive = alive && L.status == TW_REP_RUNNING;
                STIME(tl2);
                STADDL(K_CYC_TAIL, tl2 - tl1);
            }
            L.hash_flush();
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
            L.run_commit();
        #ifdef TW_STATS
            // (a second set of counters for heavy-inbox LP lanes alone: a hotspot
            // receiver's chain bounds its windows)
            const uint32_t pset = (LP && !ilight) ? P_COUNT : 0u;
            if (c.prof)
                for (int i = 0; i < P_COUNT; ++i)
                    __hip_atomic_fetch_add(gp(c.prof) + pset + i, (unsigned long long)L.st[i], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
            STIME(tepi0);
        #endif
            sc[SC_PENDING_MAIN * SR] = pending_main;
            if (!LP && L.status == TW_REP_RUNNING && L.live == 0) L.status = TW_REP_DONE;

            // (the compact geometry's replica lanes: curTime after the last pop is
            // the clock -- every pop sets both --, and every thread this launch
            // created took a thread id, so neither count is carried through the
            // loop in a register; neither is the launch's starting event count, in
            // any geometry but those with far runs.  Measured: C2 +3 %, the LP
            // kernels without scratch; the run geometries' allocation lost 1.4 % on
            // C3 with it, so they keep the registers)
            constexpr bool KEEP = !LP && RUNS;
            const uint64_t threads_add = (LP || KEEP) ? (uint64_t)L.d_th : (uint64_t)(L.tidc - (uint32_t)sc[SC_TIDC * SR]);
            sc[SC_NOW * SR] = (uint64_t)L.now; sc[SC_FINAL_T * SR] = (uint64_t)((LP || KEEP) ? L.final_t : L.now);
            sc[SC_SEQ * SR] = L.seq; sc[SC_TIDC * SR] = L.tidc; sc[SC_LIVE * SR] = L.live;
            sc[SC_NEAR_N * SR] = L.near_n; sc[SC_FAR_N * SR] = L.far_n;
            sc[SC_STATUS * SR] = L.status; sc[SC_MAIN_EXC * SR] = L.cg(CW_MAINEXC);
            sc[SC_FREE_N * SR] = L.free_n; sc[SC_FTOP * SR] = L.ftop; sc[SC_BUMP * SR] = L.bump;
            sc[SC_TMO_CTR * SR] = L.cg(CW_TMO);
            if constexpr (!LP) sc[SC_TRACE_N * SR] = L.cg(CW_TRN);
            // (LP lanes: the sums below as no-return atomics, without the drain
            // above, measured slower -- C5 1,366 -> 1,448 ms, C4 7.05 -> 7.30 ms:
            // round 6, profiles/r06c/ab_lp_epi_*)
            if constexpr (KEEP) sc[SC_EVENTS * SR] = events0 + L.d_ev;
            else sc[SC_EVENTS * SR] += L.d_ev;
            if (LP) {
                sc[SC_DUE_H * SR] = L.dg(DW_HN) & 0xFFFFu;
                if (L.dg(DW_IB) >> 31)  // sent records straight into inboxes (Lane::emit)
                    min_hot((uint64_t GAS*)(PRW ? rw_at(c, RW_WIN, r) : gp(c.win) + WN_REC_MIN), (uint64_t)(te + 1));
            }
            sc[SC_DELIVERED * SR] += L.cg(CW_DL); sc[SC_DROPPED * SR] += L.cg(CW_DR);
            sc[SC_UNDELIV * SR] += L.cg(CW_UD); sc[SC_THREADS * SR] += threads_add;
            if (HR && c.Cr) {
                const uint4 ix4 = *L.rqp(RQ_IDX);
        #pragma unroll
                for (int j = 0; j < TW_RUNS; ++j) {
                    sc[(SC_RH0 + j) * SR] = Lane<LP, WG, NC, RUNS, IP>::q_at(ix4, j);
                    sc[(SC_RC0 + j) * SR] = L.rqp(RQ_TAIL + j)->w;
                }
            }
            for (uint32_t i = 0, j = 0; i < NC; ++i) {
                const uint64_t k = L.nk[i * WG];
                if (k != ~0ull)
                    gp(c.near_spill)[(size_t)(j++) * R + r] = ent(L.nbase + (int64_t)(k >> 32), L.ns[i * WG], (uint32_t)k);
            }
            bool active = L.status == TW_REP_RUNNING && L.d_ev < ev_room;
            int64_t tn = INT64_MAX;
            if (L.far_dirty) L.far_min();
            if (L.near_n) tn = L.nbase + (int64_t)(L.nrk >> 32);
            if (L.fsrc >= 0 && L.fmt < tn) tn = L.fmt;
            if (active && (tn == INT64_MAX || tn > te) && !pending_main) active = false;  // parked beyond t_end
            if (LP && L.status == TW_REP_RUNNING && tn != INT64_MAX)
                min_hot(PRW ? (uint64_t GAS*)rw_at(c, RW_TICK, r) : gp(c.next_t), (uint64_t)tn);
            {   // lanes still active: one atomic per wave
                const uint64_t am = __builtin_amdgcn_ballot_w64(active);
                const uint64_t ex = __builtin_amdgcn_ballot_w64(true);
                if (am && __builtin_amdgcn_mbcnt_hi((uint32_t)(ex >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ex, 0u)) == 0)
                    __hip_atomic_fetch_add(gp(c.n_active), (uint32_t)__builtin_popcountll(am), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
            }
            if (LP) {
                // device loop: the lane is listed again by the window its next event
                // falls in (tw_lp_compact); host loop: for the next window
                const bool more = L.status == TW_REP_RUNNING && (L.live || pending_main);
                if (c.win) {
                    const int64_t wk = more ? (pending_main ? L.now : tn) : INT64_MAX;
                    gp(c.wake)[r] = wk;
                    // per-replica windows: the lane's chunk keeps a lower bound of its wakes
                    if (PRW && wk != INT64_MAX) min_hot((uint64_t GAS*)gp(c.cw_min) + cw_idx(c, r), (uint64_t)wk);
                }
                else if (more) lp_list_next(c, r);
            }
        #ifdef TW_STATS
            {
                STIME(tepi1);
                if (c.prof)
                    __hip_atomic_fetch_add(gp(c.prof) + pset + K_CYC_EPI, (unsigned long long)(tepi1 - tepi0), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
            }
        #endif
        } while (0);
        if (!(LP && GS) || (size_t)(blk + gridDim.x) * WG >= lp_n) break;  // vmcnt(0): the last block's LDS-DMA landed before LDS is reused
    }
}


// A delivery record for local node dst: claim an inbox slot (the drain at the
// window's first tick sorts them), lower *tmin to its time, list the node for
// the next window.
__device__ __forceinline__ void lp_deliver(const Dev& c, uint4 a, uint4 b, uint64_t GAS* tmin, int64_t wend,
                                           bool upd_min) {
    const uint32_t lp = b.w - c.lp0;
    const uint32_t cap = ib_cap(c, lp);
    const uint32_t par = ib_par_in(c, cap <= TW_LIGHT);
    const uint32_t k =
        __hip_atomic_fetch_add(gp(c.inbox_n) + (size_t)par * c.R + lp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k >= cap) {
        __hip_atomic_fetch_or(gp(c.lp_err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    uint4 GAS* q = gp(c.inbox) + ((size_t)par * c.ib_total + ib_base(c, lp) + (size_t)k * ib_stride(c, cap > TW_LIGHT)) * 2;
    q[0] = a;
    q[1] = b;
    // (a record due in this window, t < wend -- a short link into a phase-1
    // node -- is drained at phase 1's first tick: it does not bound the next window)
    if (upd_min && c.rw && c.win) {  // per-replica windows: the record's replica's window and minimum
        const int64_t te = rw_tend(c, lp, gp(c.win)[WN_L]);
        if (ent_t(a) > te) min_hot((uint64_t GAS*)rw_at(c, RW_WIN, lp), (uint64_t)ent_t(a));
    } else if (upd_min && ent_t(a) >= wend) {
        min_hot(tmin, (uint64_t)ent_t(a));
    }
    // a lane whose node may hold more than TW_LIGHT records is served by
    // tw_lp_due: its first pending record lists it for the next window's pass
    // (device loop; the list of window wid + 1)
    if (k == 0 && cap > TW_LIGHT && c.win) {
        const uint32_t l = (c.wid + 1u) & 1u;
        const uint32_t i = __hip_atomic_fetch_add(gp(c.heavy_n) + l, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (i < c.R) gp(c.heavy)[(size_t)l * c.R + i] = lp;  // (once per lane and list: a guard, not a limit)
        else __hip_atomic_fetch_or(gp(c.lp_err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    lp_list_next(c, lp);
}
// Batched LP: a spawn record pair (Lane::emit_spawn) for a local lane.
__device__ __forceinline__ void lp_spawn(const Dev& c, const uint4 GAS* o, uint64_t GAS* tmin) {
    const uint4 a = o[0], b = o[1], d = o[2], e = o[3];
    const uint32_t dst = b.w;
    if (dst < c.lp0 || dst >= c.lp0 + c.R) {
        __hip_atomic_fetch_or(gp(c.lp_err), 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    const uint32_t lp = dst - c.lp0;
    const uint32_t k = __hip_atomic_fetch_add(gp(c.spawn_n) + lp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k >= TW_SPN) {
        __hip_atomic_fetch_or(gp(c.lp_err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    uint4 GAS* q = gp(c.spawn) + ((size_t)k * c.R + lp) * 4;
    q[0] = a;
    q[1] = b;
    q[2] = d;
    q[3] = e;
    // this tick's earliest spawn: one in the current window reruns it (tw_lp_fill),
    // with the target lane appended to the running window's work list (once)
    (void)tmin;
    // (one store / append per wave on the window's shared words: a start-up
    // window of batched C3 packs a spawn per node per replica -- 8.2M records
    // at 8,192 replicas -- and same-address writes serialise in the L2)
    if (c.rw && c.win) {  // per-replica windows: the spawn bounds its replica's next window, or reruns this one
        min_hot((uint64_t GAS*)rw_at(c, RW_TICK, lp), (uint64_t)ent_t(a));
        const bool here = ent_t(a) <= rw_tend(c, lp, gp(c.win)[WN_L]);
        const uint64_t hm = __builtin_amdgcn_ballot_w64(here);
        if (here && __builtin_amdgcn_mbcnt_hi((uint32_t)(hm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hm, 0u)) == 0)
            gp(c.win)[WN_SPN_HERE] = 1;
    } else {
        min_hot((uint64_t GAS*)(gp(c.win) + WN_SPN_MIN), (uint64_t)ent_t(a));
    }
    if (__hip_atomic_exchange(gp(c.inlist) + lp, c.wid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != c.wid) {
        const uint32_t i = wave_append(gp(c.act_n) + c.act_cur * TW_LP_NB, 1u);
        if (i < c.R) gp(c.act)[(size_t)c.act_cur * TW_LP_NB * c.R + i] = lp;  // (inlist: once per window)
        else __hip_atomic_fetch_or(gp(c.lp_err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    lp_list_next(c, lp);
}

// Delivery records -> inboxes of local nodes (or the foreign buffer for the
// host exchange).  One thread per record.
__global__ void __launch_bounds__(256) tw_lp_scatter(Dev c, const uint4* recs, uint32_t n, uint4* foreign,
                                                     uint32_t* n_foreign, uint32_t foreign_cap) {
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint4 a = gp(recs)[(size_t)i * 2], b = gp(recs)[(size_t)i * 2 + 1];
    uint32_t dst = b.w;
    if (dst >= c.lp0 && dst < c.lp0 + c.R) {
        lp_deliver(c, a, b, gp(c.next_t), INT64_MIN);
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

// ---- device-driven windows (tw_lp_tick / tw_lp_tick_import / tw_lp_tick_end)
// The window's state is read from c.win by every kernel; a finished loop makes
// them all return at once.
__device__ __forceinline__ bool win_enter(Dev& c) {
    const int64_t GAS* w = gp(c.win);
    if (w[WN_FLAGS] & WN_DONE) return false;
    c.act_cur = (uint32_t)w[WN_ACT];
    c.wid = (uint32_t)w[WN_WID];
    return true;
}
// this tick's records: local ones into inboxes, foreign ones into the send
// block of their owner rank (starts[g] <= dst < starts[g + 1]).  Blocks are
// `stride` records apart; this tick sends the first `cap` of each (the size
// the ranks agreed on, <= stride).  A block's header counts every record
// meant for that rank (the demand, reduced as RD_DEMAND); records beyond cap
// wait in the carry buffer for the next tick, which keeps the window running
// (lp_fill).  The previous tick's carry goes first: tw_lp_pack_carry claims
// its block slots in a launch of its own before tw_lp_pack's outbox loop.  A
// carry that outgrows its capacity (demand above the agreed block size for
// many ticks in a row: the block size follows the demand every 16 ticks) is
// lp_err bit 8, which stops every rank at the same tick.
__device__ __forceinline__ void lp_foreign(const Dev& c, uint4 a, uint4 b, uint4* send, const uint32_t* starts,
                                           uint32_t world, uint32_t stride, uint32_t cap, uint32_t cout) {
    const uint32_t dst = b.w;
    uint32_t lo = 0, hi = world;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (gp(starts)[mid] <= dst) lo = mid; else hi = mid;
    }
    uint4 GAS* blk = gp(send) + (size_t)lo * (stride + 1) * 2;
    const uint32_t k = __hip_atomic_fetch_add((uint32_t GAS*)blk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k < cap) {
        blk[(size_t)(k + 1) * 2] = a;
        blk[(size_t)(k + 1) * 2 + 1] = b;
        return;
    }
    const uint32_t j = __hip_atomic_fetch_add(gp(c.carry_n) + cout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (j >= c.carry_cap) {
        __hip_atomic_fetch_or(gp(c.lp_err), 8u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    uint4 GAS* q = gp(c.carry) + ((size_t)cout * c.carry_cap + j) * 2;
    q[0] = a;
    q[1] = b;
}
// The records the previous tick's blocks had no room for claim this tick's
// block slots first (multi-rank exchanges only; launched before tw_lp_pack)
__global__ void __launch_bounds__(256) tw_lp_pack_carry(Dev c, uint4* send, const uint32_t* starts, uint32_t world,
                                                        uint32_t stride, uint32_t cap) {
    if (!win_enter(c) || !c.carry || !send || world <= 1) return;
    // carry buffers by tick parity: read the previous tick's, write this one's
    const uint32_t tk = (uint32_t)gp(c.win)[WN_TICKS], cout = tk & 1u, cin = cout ^ 1u;
    uint32_t nc = *gp(c.carry_n + cin);
    nc = nc < c.carry_cap ? nc : c.carry_cap;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < nc; i += gridDim.x * 256) {
        const uint4 GAS* q = gp(c.carry) + ((size_t)cin * c.carry_cap + i) * 2;
        lp_foreign(c, q[0], q[1], send, starts, world, stride, cap, cout);
    }
}
__global__ void __launch_bounds__(256) tw_lp_pack(Dev c, uint4* send, const uint32_t* starts, uint32_t world,
                                                  uint32_t stride, uint32_t cap) {
    if (!win_enter(c)) return;
    uint32_t n = *gp(c.out_n);
    n = n < c.out_cap ? n : c.out_cap;
    uint64_t GAS* tmin = (uint64_t GAS*)(gp(c.win) + WN_REC_MIN);
    const int64_t wend = gp(c.win)[WN_T] + gp(c.win)[WN_L];
    const uint32_t cout = (uint32_t)gp(c.win)[WN_TICKS] & 1u;  // this tick's carry buffer
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const uint4 a = gp(c.outbox)[(size_t)i * 2], b = gp(c.outbox)[(size_t)i * 2 + 1];
        const uint32_t dst = b.w;
        if (b.y == TW_SPAWN_CONT) continue;  // second half of a spawn pair
        if (b.y == TW_SPAWN_KIND) {
            lp_spawn(c, gp(c.outbox) + (size_t)i * 2, tmin);
            continue;
        }
        if (dst >= c.lp0 && dst < c.lp0 + c.R) {
            lp_deliver(c, a, b, tmin, wend);
        } else if (send && world > 1 && c.carry) {
            lp_foreign(c, a, b, send, starts, world, stride, cap, cout);
        } else {
            __hip_atomic_fetch_or(gp(c.lp_err), 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}
// the records other ranks sent this tick (the first min(count, cap) of each block)
__global__ void __launch_bounds__(256) tw_lp_import(Dev c, const uint4* recv, uint32_t world, uint32_t stride,
                                                    uint32_t cap) {
    if (!win_enter(c)) return;
    uint64_t GAS* tmin = (uint64_t GAS*)(gp(c.win) + WN_REC_MIN);
    const int64_t wend = gp(c.win)[WN_T] + gp(c.win)[WN_L];
    const uint32_t total = world * cap;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
        const uint32_t g = i / cap, k = i - g * cap;
        const uint4 GAS* blk = gp(recv) + (size_t)g * (stride + 1) * 2;
        const uint32_t cnt = blk[0].x;
        if (k >= (cnt < cap ? cnt : cap)) continue;
        const uint4 a = blk[(size_t)(k + 1) * 2], b = blk[(size_t)(k + 1) * 2 + 1];
        if (b.w >= c.lp0 && b.w < c.lp0 + c.R) lp_deliver(c, a, b, tmin, wend);  // (import)
        else __hip_atomic_fetch_or(gp(c.lp_err), 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
// red = {this rank's next event time (lanes' queues, records delivered this
// window), -(lanes still active in the window), -(this rank's overflow bits),
// -(its largest per-rank record demand this tick)}, for an all-reduce(min):
// an overflow on any rank ends every rank's loop at the same tick
// (tw_lp_ctl), so no rank is left waiting in a collective
__device__ __forceinline__ void lp_fill(const Dev& c, int64_t* red, const uint4* send, uint32_t world,
                                        uint32_t stride) {
    const int64_t GAS* w = gp(c.win);
    gp(red)[RD_ERR] = -(int64_t)*gp(c.lp_err);
    uint32_t dem = 0;
    for (uint32_t g = 0; send && g < world; ++g) {
        const uint32_t k = gp(send)[(size_t)g * (stride + 1) * 2].x;
        dem = k > dem ? k : dem;
    }
    gp(red)[RD_DEMAND] = -(int64_t)dem;
    if (w[WN_FLAGS] & WN_DONE) {
        gp(red)[RD_NEXT] = INT64_MAX;
        gp(red)[RD_ACTIVE] = 0;
        return;
    }
    const uint64_t a = *gp(c.next_t), b = (uint64_t)w[WN_REC_MIN], p = *gp(c.pend_min), sp = (uint64_t)w[WN_SPN_MIN];
    const uint64_t sl = (uint64_t)w[WN_SLEEP_MIN];  // lanes not listed in this window
    uint64_t m = a < b ? a : b;
    m = p < m ? p : m;
    m = sp < m ? sp : m;
    m = sl < m ? sl : m;
    gp(red)[RD_NEXT] = m >= (uint64_t)INT64_MAX ? INT64_MAX : (int64_t)m;
    // a child forked onto another node inside this window keeps the window
    // (phase) running: its lane starts it at the next tick; so do records
    // still waiting in the exchange carry
    bool spawn_here = sp < (uint64_t)(w[WN_T] + w[WN_L]);
    if (c.rw) {  // per-replica windows: the replicas' own minima decide (tw_lpb_rctl)
        gp(red)[RD_NEXT] = 0;
        spawn_here = w[WN_SPN_HERE] != 0;
    }
    const bool carried = c.carry && *gp(c.carry_n + ((uint32_t)w[WN_TICKS] & 1u)) != 0;
    gp(red)[RD_ACTIVE] = -(int64_t)*gp(c.n_active) - (spawn_here ? 1 : 0) - (carried ? 1 : 0);
}
__global__ void tw_lp_fill(Dev c, int64_t* red, const uint4* send, uint32_t world, uint32_t stride) {
    lp_fill(c, red, send, world, stride);
}
// advance: every rank idle in this window -> T := the global next time (a
// fresh window: flip the work lists), else rerun the window
// (one rank: the reduction words are this rank's own, filled here -- one
// launch per tick fewer than tw_lp_fill + tw_lp_ctl)
__global__ void tw_lp_ctl(Dev c, int64_t* red, uint4* send, uint32_t world, uint32_t stride, uint32_t filled) {
    if (!filled) lp_fill(c, red, nullptr, 1, 0);
    int64_t GAS* w = gp(c.win);
    if (w[WN_FLAGS] & WN_DONE) return;
    w[WN_TICKS] += 1;
    // the carry buffer the next tick writes (this tick's pack read it)
    if (c.carry) gp(c.carry_n)[(uint32_t)w[WN_TICKS] & 1u] = 0;
    const int64_t dem = -gp(red)[RD_DEMAND];
    w[WN_XMAX] = dem > w[WN_XMAX] ? dem : w[WN_XMAX];
    *gp(c.out_n) = 0;
    for (uint32_t g = 0; send && g < world; ++g) gp(send)[(size_t)g * (stride + 1) * 2].x = 0;
    *gp(c.n_active) = 0;
    *gp(c.next_t) = ~0ull;
    w[WN_SPN_MIN] = (int64_t)~0ull;
    w[WN_SPN_HERE] = 0;
    if (gp(red)[RD_ERR] < 0) {  // some rank overflowed: every rank stops here (tw_lp_progress reports it)
        *gp(c.lp_err) |= (uint32_t)(-gp(red)[RD_ERR]) | 16u;
        w[WN_FLAGS] = WN_DONE;
        w[WN_STEP] = RS_STOP;
        return;
    }
    if (gp(red)[RD_ACTIVE] < 0) {  // rerun this phase of the window
        w[WN_FLAGS] &= ~(WN_FRESH | WN_PH1FRESH);
        w[WN_STEP] = RS_RERUN;
        return;
    }
    if (c.has_ph1 && w[WN_PHASE] == 0) {
        // phase 0 is done with the window: phase 1 (the nodes fed by short
        // links) runs it now; the phase-0 nodes' next time waits in WN_NT0
        w[WN_PHASE] = 1;
        w[WN_NT0] = gp(red)[RD_NEXT];
        w[WN_FLAGS] = WN_PH1FRESH;
        w[WN_STEP] = RS_PHASE1;
        return;
    }
    w[WN_WINDOWS] += 1;
    int64_t t = gp(red)[RD_NEXT];
    if (w[WN_PHASE]) t = w[WN_NT0] < t ? w[WN_NT0] : t;
    w[WN_PHASE] = 0;
    w[WN_STEP] = RS_ADVANCE;
    w[WN_REPS] = 0;  // (per-replica windows: tw_lpb_rctl counts the replicas still running)
    if (t == INT64_MAX) {
        w[WN_T] = INT64_MAX;
        w[WN_FLAGS] = WN_DONE;
        return;
    }
    w[WN_T] = t;
    const uint32_t act = (uint32_t)w[WN_ACT] ^ 1u;
    w[WN_ACT] = act;
    w[WN_WID] += 1;
    // tw_lp_due serves heavy list wid & 1 now; the other one collects this window's
    *gp(c.pend_min) = ~0ull;
    gp(c.heavy_n)[(w[WN_WID] + 1) & 1] = 0;
    for (int k = 0; k < TW_LP_NB; ++k) gp(c.act_n)[act * TW_LP_NB + k] = 0;  // tw_lp_compact builds it next
    w[WN_REC_MIN] = (int64_t)~0ull;
    w[WN_SLEEP_MIN] = INT64_MAX;  // tw_lp_compact recomputes it for the new window
    w[WN_FLAGS] = WN_FRESH;
}
// Per-replica windows (batched LP, Dev::rw): this tick's decision of
// tw_lp_ctl applied to every replica's own window -- a rerun keeps it, phase 1
// keeps phase 0's next time, an advance moves the replica's window to its own
// next event (the minimum of its lanes' next events, records, pending records
// and sleeping lanes) and counts the replicas that still have one.
__global__ void __launch_bounds__(256) tw_lpb_rctl(Dev c) {
    int64_t GAS* w = gp(c.win);
    if (w[WN_FLAGS] & WN_DONE) return;
    const uint32_t q = blockIdx.x * 256 + threadIdx.x;
    const size_t nrep = (size_t)1 << c.rep_lg;
    const int64_t step = w[WN_STEP];
    bool live = false;
    if (q < nrep) {
        uint64_t GAS* rw = (uint64_t GAS*)gp(c.rw);
        const uint64_t tk = rw[RW_TICK * nrep + q];
        rw[RW_TICK * nrep + q] = ~0ull;
        if (step == RS_PHASE1) {
            const uint64_t wn = rw[RW_WIN * nrep + q];
            rw[RW_NT0 * nrep + q] = tk < wn ? tk : wn;
        } else if (step == RS_ADVANCE && (int64_t)rw[RW_T * nrep + q] != INT64_MAX) {
            uint64_t t = rw[RW_WIN * nrep + q];
            t = tk < t ? tk : t;
            // the replica's lanes' next events: the minimum over its chunks
            const uint32_t nk = ((c.R >> c.rep_lg) + (1u << TW_CHUNK_LG) - 1u) >> TW_CHUNK_LG;
            const uint64_t GAS* cm = (const uint64_t GAS*)gp(c.cw_min) + q;
#pragma unroll 16
            for (uint32_t k = 0; k < nk; ++k) {
                const uint64_t v = cm[(size_t)k * nrep];
                t = v < t ? v : t;
            }
            if (c.has_ph1) {  // the window ran phase 1 last: phase 0's next time joins
                const uint64_t n0 = rw[RW_NT0 * nrep + q];
                t = n0 < t ? n0 : t;
            }
            rw[RW_NT0 * nrep + q] = ~0ull;
            rw[RW_WIN * nrep + q] = ~0ull;
            live = t < (uint64_t)INT64_MAX;
            rw[RW_T * nrep + q] = live ? t : (uint64_t)INT64_MAX;
        }
    }
    const uint64_t m = __builtin_amdgcn_ballot_w64(live);
    if (m && __lane_id() == (uint32_t)__builtin_ctzll(m))
        __hip_atomic_fetch_add((unsigned long long GAS*)(w + WN_REPS), (unsigned long long)__builtin_popcountll(m),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// ... and the loop ends once an advance leaves no replica running
__global__ void tw_lpb_fin(Dev c) {
    int64_t GAS* w = gp(c.win);
    if ((w[WN_FLAGS] & WN_DONE) || w[WN_STEP] != RS_ADVANCE || w[WN_REPS] != 0) return;
    w[WN_T] = INT64_MAX;
    w[WN_FLAGS] = WN_DONE;
}
// Per-replica windows: the window's work list.  One wavefront per tile of 64
// replicas x one chunk of 64 nodes, a lane per replica: a chunk is read only
// where its replica's lanes were marked (records, spawns) in the previous
// window or its lower bound of their next events falls in the replica's new
// window; a due chunk's bound is recomputed from its unlisted lanes (the listed
// ones add theirs when they run).  Lanes are appended node by node, so a
// wavefront of the event kernel gets 64 replicas of one node.
__global__ void __launch_bounds__(256) tw_lpb_compact(Dev c) {
    const int64_t GAS* w = gp(c.win);
    const int64_t fl = w[WN_FLAGS];
    if (!(fl & WN_FRESH) || (fl & WN_DONE)) return;
    const uint32_t mark = (uint32_t)w[WN_WID] - 1u, dst = (uint32_t)w[WN_ACT];
    const int64_t L = w[WN_L];
    const uint32_t nrep = 1u << c.rep_lg, nloc = c.R >> c.rep_lg;
    const uint32_t tile = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t ngrp = (nrep + 63) >> 6;
    const uint32_t k = tile / ngrp, q = (tile - k * ngrp) * 64 + __lane_id();
    if ((k << TW_CHUNK_LG) >= nloc) return;  // (wave-uniform)
    const bool have = q < nrep;
    const size_t ci = ((size_t)k << c.rep_lg) + q;
    const int64_t te = have ? rw_tend(c, q, L) : INT64_MIN;
    const int64_t cmv = have ? gp(c.cw_min)[ci] : INT64_MAX;
    const bool due = have && cmv <= te;
    const bool mk = have && gp(c.cw_mark)[ci] == mark;
    if (!__builtin_amdgcn_ballot_w64(due || mk)) return;
    // pass 1: which of the column's lanes are listed (a bit per node)
    int64_t nm = INT64_MAX;
    uint64_t bits = 0;
    const uint32_t n0 = k << TW_CHUNK_LG;
    const uint32_t nn = n0 + (1u << TW_CHUNK_LG) < nloc ? 1u << TW_CHUNK_LG : nloc - n0;
    if (due || mk) {
        // (16 nodes' words in flight at a time: one after another, the 64
        // nodes of a chunk were 64 dependent round trips per tile)
        for (uint32_t jb = 0; jb < nn; jb += 16) {
            uint32_t ls[16];
            int64_t wks[16];
#pragma unroll
            for (uint32_t i = 0; i < 16; ++i) {
                const uint32_t j = jb + i;
                const uint32_t r = ((n0 + (j < nn ? j : 0u)) << c.rep_lg) | q;
                ls[i] = (mk && j < nn) ? gp(c.listed)[r] : ~mark;
                wks[i] = (due && j < nn) ? gp(c.wake)[r] : INT64_MAX;
            }
#pragma unroll
            for (uint32_t i = 0; i < 16; ++i) {
                const uint32_t j = jb + i;
                const bool b = j < nn && ((mk && ls[i] == mark) || (due && wks[i] <= te));
                if (due && j < nn && !b && wks[i] < nm) nm = wks[i];
                bits |= (uint64_t)b << (j & 63u);
            }
        }
    }
    // pass 2: one append per tile, then node-major positions
    uint32_t tot = (uint32_t)__builtin_popcountll(bits);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) tot += __shfl_xor(tot, d, 64);
    if (tot) {
        uint32_t base = 0;
        if (__lane_id() == 0)
            base = __hip_atomic_fetch_add(gp(c.act_n) + dst * TW_LP_NB, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
        uint32_t GAS* act = gp(c.act) + (size_t)dst * TW_LP_NB * c.R;
        for (uint32_t j = 0; j < nn; ++j) {
            const bool b = (bits >> j) & 1u;
            const uint64_t m = __builtin_amdgcn_ballot_w64(b);
            if (b) {
                const uint32_t r = ((n0 + j) << c.rep_lg) | q;
                act[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = r;
                if (c.inlist) gp(c.inlist)[r] = mark + 1u;
            }
            base += (uint32_t)__builtin_popcountll(m);
        }
    }
    if (due) gp(c.cw_min)[ci] = nm;
}

// The window's work list: every node marked during the previous window
// (listed[r] == mark), split into TW_LP_NB buckets by the node's pending
// delivery records (min(inbox_n, NB-1): a wave runs until its busiest lane is
// done, so lanes with alike work share waves), in node order inside each
// block of TW_CPT * 256 nodes (so the lanes' [field][node] state accesses
// coalesce); one atomic per block and bucket claims its span.  Device loop
// (c.win): only at a window's first tick, with mark/list from the window words.
#ifndef TW_CPT
#define TW_CPT 4
#endif
__global__ void __launch_bounds__(256) tw_lp_compact(Dev c, uint32_t mark, uint32_t dst) {
    int64_t tend = INT64_MIN;  // device loop: lanes whose next event is due in the window are listed too
    int64_t L = 0;
    if (c.win) {
        const int64_t GAS* w = gp(c.win);
        const int64_t fl = w[WN_FLAGS];
        if (!(fl & WN_FRESH) || (fl & WN_DONE)) return;
        mark = (uint32_t)w[WN_WID] - 1u;
        dst = (uint32_t)w[WN_ACT];
        L = w[WN_L];
        tend = w[WN_T] + L - 1;
    }
    // per-replica windows: each lane's own replica window, and the sleeping
    // lanes' minimum per replica (every block is scanned: a block's summary
    // mixes 256 replicas)
    const bool prw = c.win && c.rw;
    static_assert(1 << TW_SUB_LG == 256, "a scan block is one pass of the workgroup");
    __shared__ unsigned long long smin;
    __shared__ unsigned long long sbm[TW_CPT][4];  // per scan block and wave: min unlisted wake
    __shared__ uint32_t sbl[TW_CPT][4];            // per scan block and wave: lanes listed
    if (threadIdx.x == 0) smin = ~0ull;
    __syncthreads();
    unsigned long long mymin = ~0ull;
    __shared__ uint32_t cnt[TW_LP_NB][TW_CPT * 4];
    __shared__ uint32_t base[TW_LP_NB];
    const uint32_t wv = threadIdx.x >> 6;
    const size_t r0 = (size_t)blockIdx.x * TW_CPT * 256 + threadIdx.x;
    const uint32_t sb0 = blockIdx.x * TW_CPT;
    __shared__ uint32_t sbs[TW_CPT];  // the block was scanned
    uint32_t key[TW_CPT];
#pragma unroll
    for (int i = 0; i < TW_CPT; ++i) {
        const size_t r = r0 + (size_t)i * 256;
        // device loop: a 256-lane block none of whose lanes was marked, listed
        // last window or due now is skipped; its unlisted minimum still counts
        bool scan = true;
        const size_t rb = (size_t)(sb0 + i) << TW_SUB_LG;  // the block's first lane
        if (c.win) {
            scan = rb < c.R;
            if (scan && !prw) {
                const uint32_t sb = sb0 + (uint32_t)i;
                const int64_t bm = gp(c.sb_min)[sb];
                scan = gp(c.sb_mark)[sb] == mark || gp(c.sb_scan)[sb] == mark || bm <= tend;
                if (!scan && bm != INT64_MAX) mymin = (unsigned long long)bm < mymin ? (unsigned long long)bm : mymin;
            }
        }
        if (threadIdx.x == 0) sbs[i] = scan;
        bool b = false;
        unsigned long long um = ~0ull;
        if (scan) {
            b = r < c.R && gp(c.listed)[r] == mark;
            if (c.win && r < c.R) {
                const int64_t wk = gp(c.wake)[r];
                b = b || wk <= (prw ? rw_tend(c, (uint32_t)r, L) : tend);
                if (!b && wk != INT64_MAX) {
                    if (prw) min_hot((uint64_t GAS*)rw_at(c, RW_WIN, (uint32_t)r), (uint64_t)wk);
                    else um = (unsigned long long)wk;
                }
            }
        }
        if (c.win && scan) {
            mymin = um < mymin ? um : mymin;
            // the block's summary for the next window: its unlisted minimum, and
            // whether it lists lanes (they run now and move their wakes)
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) {
                const unsigned long long o = __shfl_xor(um, d, 64);
                um = o < um ? o : um;
            }
            const uint64_t lb = __builtin_amdgcn_ballot_w64(b);
            if (__lane_id() == 0) {
                sbm[i][wv] = um;
                sbl[i][wv] = lb != 0;
            }
        }
        const uint32_t n_in = (TW_LP_NB > 1 && b) ? gp(c.inbox_n)[r] : 0u;
        key[i] = b ? (n_in < TW_LP_NB - 1 ? n_in : TW_LP_NB - 1) : 0xFFu;
#pragma unroll
        for (int k = 0; k < TW_LP_NB; ++k) {
            const uint64_t m = __builtin_amdgcn_ballot_w64(key[i] == (uint32_t)k);
            if (__lane_id() == 0) cnt[k][i * 4 + wv] = (uint32_t)__builtin_popcountll(m);
        }
    }
    if (mymin != ~0ull) atomicMin(&smin, mymin);
    __syncthreads();
    if (c.win && threadIdx.x < TW_CPT && sbs[threadIdx.x]) {
        const uint32_t i = threadIdx.x;
        unsigned long long m = sbm[i][0];
        for (int k = 1; k < 4; ++k) m = sbm[i][k] < m ? sbm[i][k] : m;
        gp(c.sb_min)[sb0 + i] = m == ~0ull ? INT64_MAX : (int64_t)m;
        if (sbl[i][0] | sbl[i][1] | sbl[i][2] | sbl[i][3]) gp(c.sb_scan)[sb0 + i] = mark + 1u;
    }
    if (threadIdx.x == 0 && smin != ~0ull)
        __hip_atomic_fetch_min((unsigned long long GAS*)(gp(c.win) + WN_SLEEP_MIN), smin, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x < TW_LP_NB) {
        const uint32_t k = threadIdx.x;
        uint32_t run = 0;
        for (int j = 0; j < TW_CPT * 4; ++j) {
            const uint32_t n = cnt[k][j];
            cnt[k][j] = run;
            run += n;
        }
        base[k] = run ? __hip_atomic_fetch_add(gp(c.act_n) + dst * TW_LP_NB + k, run, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)
                      : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TW_CPT; ++i) {
#pragma unroll
        for (int k = 0; k < TW_LP_NB; ++k) {
            const uint64_t m = __builtin_amdgcn_ballot_w64(key[i] == (uint32_t)k);
            if (key[i] == (uint32_t)k) {
                const uint32_t below =
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                gp(c.act)[((size_t)dst * TW_LP_NB + k) * c.R + base[k] + cnt[k][i * 4 + wv] + below] =
                    (uint32_t)(r0 + (size_t)i * 256);
                if (c.inlist) gp(c.inlist)[r0 + (size_t)i * 256] = mark + 1u;
            }
        }
    }
}
static uint32_t compact_blocks(uint32_t R) { return (R + TW_CPT * 256 - 1) / (TW_CPT * 256); }

// loop start after tw_reset: the window words; the first window's list
// (every node: tw_reset marks them all 0) is compacted next
__global__ void tw_lp_begin(Dev c, int64_t lookahead) {
    int64_t GAS* w = gp(c.win);
    w[WN_T] = 0;
    w[WN_L] = lookahead;
    w[WN_REC_MIN] = (int64_t)~0ull;
    w[WN_WINDOWS] = 0;
    w[WN_TICKS] = 0;
    w[WN_FLAGS] = WN_FRESH;
    w[WN_ACT] = 1;
    w[WN_WID] = 1;
    w[WN_PHASE] = 0;
    w[WN_NT0] = INT64_MAX;
    w[WN_SPN_MIN] = (int64_t)~0ull;
    w[WN_SLEEP_MIN] = INT64_MAX;
    w[WN_XMAX] = 0;
    w[WN_SPN_HERE] = 0;
    w[WN_REPS] = 0;
    w[WN_STEP] = RS_RERUN;
    if (c.carry) gp(c.carry_n)[0] = gp(c.carry_n)[1] = 0;
    for (int k = 0; k < TW_LP_NB; ++k) gp(c.act_n)[TW_LP_NB + k] = 0;
    *gp(c.out_n) = 0;
    *gp(c.n_active) = 0;
    *gp(c.next_t) = ~0ull;
    *gp(c.pend_min) = ~0ull;
    gp(c.heavy_n)[0] = gp(c.heavy_n)[1] = 0;
}

// Heavy inboxes at a window's first tick (device loop).  A lane whose node may
// hold more than TW_LIGHT pending records (a hotspot receiver: hundreds of
// messages in flight) would otherwise hold every one of them as a phantom
// thread, with a slot, in its queue.  Here one workgroup per such lane with
// records stages them in LDS, keeps the ones due in this window [T, T + L) as
// the lane's due run, sorted by (t, link, payload, src, kind) -- rec_less, the
// order the light drain inserts them in -- with their queue seqs reserved now,
// as if they had been queued at the window's start; the rest stay in the inbox
// (their earliest time bounds the next window) and the lane is listed for the
// next window's pass.
//
// The sort is an LDS segmented radix (counting) sort by timestamp: a due
// record's key is its offset t - T < L inside the window, so one counting pass
// over L bins (histogram by LDS atomics, a workgroup scan of the bins, a
// scatter) orders the run by timestamp; each segment of equal timestamps
// (mostly 0-2 records) is then put in rec_less order by one thread.  Windows
// longer than TW_DUE_BINS use a rank-by-comparison fallback.
#define TW_DUE_GRID 1024  // tw_lp_due workgroups (each serves heavy lanes in turn)
#define TW_DUE_BINS 2048  // counting-sort bins: windows up to 2048 µs
// exclusive prefix sum of one value per thread over the 256-thread workgroup
// (a shuffle scan in each wave, then the four wave totals); *total = the sum
__device__ __forceinline__ uint32_t wg_excl_scan(uint32_t v, uint32_t* wsum, uint32_t* total) {
    const uint32_t lane = __lane_id(), wv = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        x += lane >= (uint32_t)d ? y : 0u;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    uint32_t base = 0;
    for (uint32_t k = 0; k < wv; ++k) base += wsum[k];
    *total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
    return base + x - v;
}
// A due-run record's second quad: {link, kind, src, reply link}.  Its
// destination (b.w) is the lane itself, so the slot carries link_rev[link]
// instead, looked up here off the lane's chain: DELIVER hands it to the
// handler's RLINK without a load.
__device__ __forceinline__ uint4 due_rec_b(const Dev& c, uint4 b) {
    return make_uint4(b.x, b.y, b.z, b.x < c.L ? gp(c.link_rev)[b.x] : 0u);
}

// ---------------------------------------------------------------------------
// Batched delivery of a heavy lane's due run (round 5, Dev::lpc_bat).  A
// hotspot receiver (bench/Network Receiver/Main.hs:32-38) gets ~256 pings per
// 1-ms window, and the event kernel runs them one after the other on the
// lane's chain (a due pop, DELIVER, the handler's passes, the send's record:
// ≈ 23 µs per message).  When a record's handler is batchable
// (classify_batch: its effects are its own) and no other event of the lane
// falls between the record's events, the record runs here instead, one per
// thread of tw_lp_due's workgroup, with the totals the sequential loop reaches.

// One due record as the event kernel handles it: the deliverer's wake (a
// phantom pop, counted by the sender); DELIVER's binding check (Lane::pass
// TW_OP_DELIVER) -- undeliverable, or the fork_ of the handler: the
// deliverer's resume at t + 1 on the sending node and the handler's first pop
// at t (TimedT.hs:326-342, MonadDialog.hs:317); the handler's code (the hot
// classes of Lane::pass; TW_OP_SEND's LP branch); the resume of the send's
// 1-µs yield, whose instruction is END.  ok = 0: the record runs on the chain.
// The effects beyond the lane itself come back as data (due_effects makes
// them): the deliverer's resume term on the sending node, the send's record.
struct DueX {
    uint32_t ok, yld, dl, ud, dr, ev, th, sq;
    int64_t fin, last;  // final_t candidate, the lane's clock after the record
    uint64_t h;         // terms of the lane's own node
    uint64_t hs;        // the term of the sending node (0: none or the lane's own)
    uint32_t hs_lane;   // its lane
    uint32_t lk, k2, dst;  // the send's record (yld): link, kind, destination lane
    int64_t ta, pay;
    uint4 dh;
};
// Lane::emit for a record of the batch (the thread's own append: no wave
// aggregation); returns 1 for a record written straight into a light inbox
__device__ __forceinline__ uint32_t due_emit(const Dev& c, uint32_t wid, int64_t ta, int64_t payload, uint32_t link,
                                             uint32_t kind, uint32_t src, uint32_t dst, uint4 dh, bool defer = false) {
    const uint4 q0 = make_uint4((uint32_t)ta, (uint32_t)((uint64_t)ta >> 32), (uint32_t)payload,
                                (uint32_t)((uint64_t)payload >> 32));
    const uint4 q1 = make_uint4(link, kind, src, dst);
    if (c.dpar && c.win && !(dh.x >> 31) && dst - c.lp0 < c.R) {
        const uint32_t lp = dst - c.lp0;
        const uint32_t par = (wid + 1u) & 1u;
        const uint32_t k = __hip_atomic_fetch_add(gp(c.inbox_n) + (size_t)par * c.R + lp, 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
        if (k >= dh.z) {
            __hip_atomic_fetch_or(gp(c.lp_err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return 0u;
        }
        const size_t base = c.ib_off ? ((size_t)dh.y << c.rep_lg) + (dst & ((1u << c.rep_lg) - 1u)) : (size_t)lp;
        uint4 GAS* q = gp(c.inbox) + ((size_t)par * c.ib_total + base + (size_t)k * ib_stride(c, false)) * 2;
        q[0] = q0;
        q[1] = q1;
        if (defer) {  // (tw_lp_due_batch runs before the window's list is built: tw_lp_dmark marks it after)
            const uint32_t j = __hip_atomic_fetch_add(gp(c.dmk_n) + (wid & 1u), 1u, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
            if (j < c.dmk_cap) gp(c.dmk)[(size_t)(wid & 1u) * c.dmk_cap + j] = lp;
            else __hip_atomic_fetch_or(gp(c.lp_err), 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            lp_mark(c, lp, wid);
        }
        return 1u;
    }
    const uint32_t i = __hip_atomic_fetch_add(gp(c.out_n), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (i >= c.out_cap) {
        __hip_atomic_fetch_or(gp(c.lp_err), 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0u;
    }
    uint4 GAS* o = gp(c.outbox) + (size_t)i * 2;
    o[0] = q0;
    o[1] = q1;
    return 0u;
}
// (the program image, constant pool, listener table and its batchable flags
// staged in LDS by tw_lp_batch: BP)
struct BProg {
    const uint2 LAS* P;
    const int64_t LAS* K;
    const uint32_t LAS* LPC;
    const uint8_t LAS* BAT;
};
__device__ DueX due_exec(const Dev& c, const BProg& bp, uint32_t r, uint32_t set, uint4 a, uint4 b) {
    DueX o{};
    o.hs_lane = 0xFFFFFFFFu;
    const int64_t t = ent_t(a);
    const int64_t payload = (int64_t)(((uint64_t)a.w << 32) | a.z);
    const uint32_t link = b.x, kind = b.y, src = b.z;
    const uint32_t node = (c.lp0 + r) >> c.rep_lg, rho = (c.lp0 + r) & ((1u << c.rep_lg) - 1u);
    o.last = t;
    o.fin = INT64_MIN;
    uint32_t lpc = TW_PC_NONE;
    size_t e = 0;
    if (set && kind < c.n_kinds) {
        e = (size_t)(set - 1u) * c.n_kinds + kind;
        lpc = bp.LPC[e];
    }
    if (lpc == TW_PC_NONE) {  // no listener: undeliverable, the phantom deliverer ends
        o.ok = 1;
        o.ud = 1;
        o.h = term(t, TW_KIND_UNDELIV | kind, payload);
        return o;
    }
    if ((lpc & TW_LPC_INLINE) || !bp.BAT[e]) return o;
    o.dl = 1;
    o.ev = 2;
    o.th = 1;
    o.sq = 1;
    o.fin = t + 1;
    o.h = term(t, TW_KIND_RECV | kind, payload) + term0(t, TW_KIND_RESUME | (lpc & 0xFFFFu));
    {
        const uint64_t hs = term0(t + 1, TW_KIND_RESUME | (TW_PC_DELIVER_STUB + 2));
        if (src == node) {
            o.h += hs;
        } else {
            o.hs = hs;
            o.hs_lane = (src << c.rep_lg) | rho;
        }
    }
    int64_t rr[4] = {payload, (int64_t)link, (int64_t)src, (int64_t)kind};
    uint32_t pc = lpc & 0xFFFFu;
    for (uint32_t n = 0; n <= c.n_insns; ++n) {  // (forward control flow only: classify_batch)
        if (pc >= c.n_insns) break;
        const uint2 in = bp.P[pc];
        const uint32_t w = in.x, op = w & 0xFFu, ai = (w >> 8) & 3u, b16 = w >> 16;
        const int32_t imm = (int32_t)in.y;
        const int64_t ra = rr[ai], rb = rr[b16 & 3u];
        if (op == TW_OP_END) {
            o.ok = 1;
            return o;
        }
        uint32_t tgt = pc + 1;
        if (op == TW_OP_SEND) {
            uint64_t lk = (uint64_t)ra;
            bool lbad = false;
            const bool fz = (b16 & (TW_SEND_VIA_LINK | TW_SEND_VIA_RLINK)) != 0;
            if (b16 & TW_SEND_VIA_LINK) {
                lk = (uint64_t)((int64_t)gp(c.out_off)[node] + imm);
            } else if (b16 & TW_SEND_VIA_RLINK) {
                const uint64_t rin = (uint64_t)rr[(b16 >> 12) & 3u];
                lbad = rin >= c.L;
                // (the reply to the record's own link: link_rev[link] is the
                // due record's fourth word, due_rec_b -- no load)
                if (!lbad) lk = rin == (uint64_t)link ? (uint64_t)b.w : gp(c.link_rev)[rin];
            }
            if (lbad || lk >= c.L) break;  // the replica's error: the chain reports it
            const uint32_t k2 = b16 & 0xFFu, pr = (b16 >> 8) & 3u;
            const int64_t pay = (fz && pr == ai) ? (int64_t)lk : rr[pr];
            tgt = fz ? pc + 2 : pc + 1;
            if (tgt >= c.n_insns || (bp.P[tgt].x & 0xFFu) != TW_OP_END) break;
            const uint32_t ent = c.link_table ? gp(c.link_table)[(((size_t)lk * c.D) << c.rep_lg) + rho] : 0u;
            // (the destination entry goes out with the table entry: one round trip)
            const uint4 dh = gp(c.link_dsth)[lk];
            asm volatile("" ::"v"(dh.x));
            if (ent & TW_LINK_DROP) {  // dropped: the handler goes on to its END at t
                o.dr += 1;
                o.h += term(t, TW_KIND_DROP | k2, pay);
                pc = tgt;
                continue;
            }
            const int64_t dly = (int64_t)(ent & 0x7FFFFFFFu) + tx_us(c, lk, k2);
            if (dly < c.lookahead) break;  // (no two-phase windows with lpc_bat)
            const int64_t ta = t + dly;
            o.h += term0(t, TW_KIND_RESUME | TW_PC_DELIVER_STUB) + term0(ta, TW_KIND_RESUME | (TW_PC_DELIVER_STUB + 1));
            o.ev += 2;
            o.th += 1;
            o.fin = ta > o.fin ? ta : o.fin;
            o.dh = dh;
            o.lk = (uint32_t)lk;
            o.k2 = k2;
            o.dst = ((o.dh.x & 0x7FFFFFFFu) << c.rep_lg) | rho;
            o.ta = ta;
            o.pay = pay;
            // the send's 1-µs yield (a fork: TimedT.hs:340); the resume runs END
            o.sq += 1;
            o.ev += 1;
            o.yld = 1;
            o.h += term0(t + 1, TW_KIND_RESUME | (tgt & 0xFFFFu));
            o.last = t + 1;
            o.ok = 1;
            return o;
        }
        const uint32_t f = uop_insn(w);
        if ((f & (U_FX | U_NS)) || U_TK(f) != TK_NONE) break;  // (not admitted by classify_batch)
        const uint32_t ak = U_ALU(f), ld = U_LD(f), jm = U_JM(f);
        bool wr = false;
        int64_t v = 0;
        if (ak != A_NONE) {
            if (ak == A_TID) break;
            v = ak == A_IMM ? (int64_t)imm : ak == A_K ? bp.K[imm] : ak == A_ADDI ? ra + (int64_t)imm
                : ak == A_MULI ? ra * (int64_t)imm : ak == A_MOV ? rb : ak == A_ADD ? ra + rb
                : ak == A_SUB ? ra - rb : ak == A_NOW ? t : (int64_t)node;
            wr = true;
        }
        if (ld == LD_NV) {
            v = gp(c.nvars)[(size_t)(b16 & 3u) * c.R + r];
            wr = true;
        } else if (ld == LD_OUT) {
            v = (int64_t)gp(c.out_off)[node] + imm;
            wr = true;
        } else if (ld == LD_RL) {
            if ((uint64_t)rb >= c.L) break;
            v = rb == (int64_t)link ? (int64_t)b.w : (int64_t)gp(c.link_rev)[rb];
            wr = true;
        }
        if (f & U_TR) o.h += term(t, TW_KIND_TRACE | ((uint32_t)imm & 0xFFFFu), ra);
        if (f & U_TR2) o.h += term(t, TW_KIND_TRACE | (b16 & 0x1FFFu), rr[(b16 >> 13) & 3u]);
        if (f & U_P2) tgt = pc + 2;
        if (jm != JM_NONE) {
            const int64_t bb = (int64_t)(int16_t)b16;
            const uint32_t ci = (ra == rb ? 1u : 0u) | (ra < rb ? 2u : 0u) | (ra == bb ? 4u : 0u);
            tgt = ((jm >> ci) & 1u) ? (uint32_t)imm : tgt;
        }
        if (wr) rr[ai] = v;
        pc = tgt;
    }
    o.ok = 0;  // an error or a path outside the admitted code: the chain runs it
    return o;
}
// The effects of a batched record beyond its lane (due_exec's data): the
// sending node's term, the send's record; returns 1 for a record written
// straight into a light inbox
__device__ __forceinline__ uint32_t due_effects(const Dev& c, uint32_t wid, uint32_t node, const DueX& x,
                                                bool defer = false) {
    if (x.hs_lane != 0xFFFFFFFFu)
        __hip_atomic_fetch_add((unsigned long long GAS*)(gp(c.hash_g) + x.hs_lane), (unsigned long long)x.hs,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return x.yld ? due_emit(c, wid, x.ta, x.pay, x.lk, x.k2, node, x.dst, x.dh, defer) : 0u;
}

__global__ void __launch_bounds__(256) tw_lp_due(Dev c) {
    const int64_t GAS* w = gp(c.win);
    const int64_t fl = w[WN_FLAGS];
    if (!(fl & WN_FRESH) || (fl & WN_DONE)) return;
    const uint32_t wid = (uint32_t)w[WN_WID];
    const int64_t T0 = w[WN_T], L = w[WN_L];
    const bool radix = L <= TW_DUE_BINS;
    const uint32_t nb = radix ? (uint32_t)L : 0u;
    const uint32_t lst = wid & 1u;
    uint32_t nh = gp(c.heavy_n)[lst];
    nh = nh < c.R ? nh : c.R;  // (an over-full list has set lp_err)
    __shared__ uint4 ea[TW_HEAVY_CAP], eb[TW_HEAVY_CAP];
    __shared__ uint16_t dix[TW_HEAVY_CAP];  // entry index of the i-th due record (arrival order)
    __shared__ uint16_t srt[TW_HEAVY_CAP];  // ... of the i-th due record in due-run order
    // counts -> segment offsets -> segment ends, two 16-bit bins per word (bin
    // b in half b & 1: every value is <= TW_HEAVY_CAP, so a half never carries
    // into the other).  Unpacked, the kernel held 24 B more than half of the
    // CU's 160 KB of LDS and ran one workgroup per CU; packed it runs two.
    __shared__ uint32_t bins[TW_DUE_BINS / 2];
    __shared__ uint32_t wsum[4];
    __shared__ unsigned long long smin;
    static_assert(TW_HEAVY_CAP == 256 * 8, "eight entries per thread");
    static_assert(TW_DUE_BINS == 256 * 8, "eight bins per thread");
    const uint32_t tid = threadIdx.x;
    const size_t st = ib_stride(c, true);  // (heavy lanes only)
    auto bsh = [](uint32_t b) { return (b & 1u) * 16u; };
    auto bget = [&](uint32_t b) { return (bins[b >> 1] >> bsh(b)) & 0xFFFFu; };
    auto binc = [&](uint32_t b) { return (atomicAdd(&bins[b >> 1], 1u << bsh(b)) >> bsh(b)) & 0xFFFFu; };
    for (uint32_t hi = blockIdx.x; hi < nh; hi += gridDim.x) {
        const uint32_t r = gp(c.heavy)[(size_t)lst * c.R + hi];
        // the lane's window: the batch's, or its replica's own (per-replica windows)
        const int64_t T = c.rw ? *rw_at(c, RW_T, r) : T0;
        if (T == INT64_MAX) continue;  // (a finished replica has no records)
        const int64_t tend = T + L - 1;
        uint32_t n = gp(c.inbox_n)[r];
        const uint32_t cap = ib_cap(c, r);
        n = n < cap ? n : cap;
        const size_t ib = ib_base(c, r);
        for (uint32_t k = tid; k < n; k += 256) {
            const uint4 GAS* q = gp(c.inbox) + (ib + (size_t)k * st) * 2;
            ea[k] = q[0];
            eb[k] = q[1];
        }
        if (tid == 0) smin = ~0ull;
        for (uint32_t i = tid; i < (nb + 1) / 2; i += 256) bins[i] = 0;
        __syncthreads();
        // thread tid owns entries [8 tid, 8 tid + 8): due flags, then a scan
        uint32_t my = 0;
        for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t k = tid * 8 + j;
            my += (k < n && ent_t(ea[k]) <= tend) ? 1u : 0u;
        }
        uint32_t nd = 0;
        uint32_t before = wg_excl_scan(my, wsum, &nd);
        // due records -> dix (arrival order) and their timestamp bins; the rest
        // compacted back into the inbox in arrival order (every record is
        // staged in LDS already)
        unsigned long long mn = ~0ull;
        for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t k = tid * 8 + j;
            if (k >= n) break;
            const int64_t t = ent_t(ea[k]);
            if (t <= tend) {
                dix[before++] = (uint16_t)k;
                if (radix) (void)binc(t > T ? (uint32_t)(t - T) : 0u);
            } else {
                uint4 GAS* q = gp(c.inbox) + (ib + (size_t)(k - before) * st) * 2;
                q[0] = ea[k];
                q[1] = eb[k];
                mn = (unsigned long long)t < mn ? (unsigned long long)t : mn;
            }
        }
        if (mn != ~0ull) atomicMin(&smin, mn);
        __syncthreads();
        if (radix) {
            // bin counts -> each bin's first position (thread tid owns bins [8 tid, 8 tid + 8))
            uint32_t cnt8[8], sum = 0;
            for (uint32_t j = 0; j < 8; ++j) {
                const uint32_t bi = tid * 8 + j;
                cnt8[j] = bi < nb ? bget(bi) : 0u;
                sum += cnt8[j];
            }
            uint32_t tot = 0;
            uint32_t off = wg_excl_scan(sum, wsum, &tot);
            for (uint32_t j = 0; j < 8; j += 2) {  // (the thread's bins are four whole words)
                const uint32_t bi = tid * 8 + j;
                const uint32_t o0 = off, o1 = off + cnt8[j];
                off = o1 + cnt8[j + 1];
                if (bi < nb) bins[bi >> 1] = o0 | (bi + 1 < nb ? o1 << 16 : 0u);
            }
            __syncthreads();
            // scatter by timestamp (positions inside a segment in any order);
            // afterwards bins[b] = the end of segment b
            for (uint32_t i = tid; i < nd; i += 256) {
                const uint32_t k = dix[i];
                const int64_t t = ent_t(ea[k]);
                const uint32_t pos = binc(t > T ? (uint32_t)(t - T) : 0u);
                srt[pos] = (uint16_t)k;
            }
            __syncthreads();
            // each segment of equal timestamps into rec_less order
            for (uint32_t bi = tid; bi < nb; bi += 256) {
                const uint32_t s0 = bi ? bget(bi - 1) : 0u, s1 = bget(bi);
                for (uint32_t x = s0 + 1; x < s1; ++x) {
                    const uint16_t k = srt[x];
                    uint32_t y = x;
                    while (y > s0 && rec_less(ea[k], eb[k], ea[srt[y - 1]], eb[srt[y - 1]])) {
                        srt[y] = srt[y - 1];
                        --y;
                    }
                    srt[y] = k;
                }
            }
            __syncthreads();
            for (uint32_t i = tid; i < nd; i += 256) {
                const uint32_t k = srt[i];
                uint4 GAS* q = gp(c.due) + (ib + (size_t)i * st) * 2;
                q[0] = ea[k];
                q[1] = due_rec_b(c, eb[k]);
            }
        } else {
            // long windows: rank of every due record among the due ones (ties by
            // arrival) = its position in the due run
            for (uint32_t i = tid; i < nd; i += 256) {
                const uint32_t k = dix[i];
                const uint4 a = ea[k], b = eb[k];
                uint32_t rank = 0;
                for (uint32_t j = 0; j < nd; ++j) {
                    const uint32_t m = dix[j];
                    rank += (rec_less(ea[m], eb[m], a, b) || (j < i && !rec_less(a, b, ea[m], eb[m]))) ? 1u : 0u;
                }
                uint4 GAS* q = gp(c.due) + (ib + (size_t)rank * st) * 2;
                q[0] = a;
                q[1] = due_rec_b(c, b);
            }
        }
        if (tid == 0) {
            const uint32_t left = n - nd;
            gp(c.inbox_n)[r] = left;
            uint64_t* sc = gp(c.scal) + (size_t)r * SC_LP_STRIDE;  // (LP: the lane's block)
            const uint64_t s0 = sc[SC_SEQ];
            if (s0 + nd >= 0xFFFFFFFFull) {
                if (sc[SC_STATUS] == TW_REP_RUNNING) sc[SC_STATUS] = TW_REP_ERR_COUNTER;
            } else {
                sc[SC_SEQ] = s0 + nd;  // the due run's queue seqs: s0 + 1 .. s0 + nd
            }
            sc[SC_DUE_SEQ] = s0;
            sc[SC_DUE_N] = nd;
            sc[SC_DUE_H] = 0;
            if (c.bat_ctr) atomicAdd(gp(c.bat_ctr) + 1, (unsigned long long)nd);
            if (smin != ~0ull)
                __hip_atomic_fetch_min(c.rw ? (uint64_t GAS*)rw_at(c, RW_WIN, r) : gp(c.pend_min), (uint64_t)smin,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // due now: this window's list (compacted next, from mark wid - 1);
            // records left for later windows: the next window's pass
            if (nd) lp_mark(c, r, wid - 1u);
            if (left) {
                const uint32_t l = lst ^ 1u;
                const uint32_t i = __hip_atomic_fetch_add(gp(c.heavy_n) + l, 1u, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
                if (i < c.R) gp(c.heavy)[(size_t)l * c.R + i] = r;
                else __hip_atomic_fetch_or(gp(c.lp_err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
    }
}


// The batch of a window's first tick, after tw_lp_due sorted the heavy lanes'
// due runs and the work list was built (the senders' inbox marks of this
// batch are for the next window's list: made before tw_lpb_compact, they would
// hide the marks it reads).  One workgroup per heavy lane at a time, the first
// TW_BATCH_CAP records of its due run staged in LDS in due-run order, the
// program tables staged once per workgroup (a program over the caps is not
// batched).  Per lane: the eligibility and the lane's next queued event; a dry
// run of every record -> the longest prefix whose records are batchable,
// precede that event, and whose resumes precede the next record's wake (a
// prefix max of the resume times); the prefix's effects (kept from the dry run
// for each thread's first record); thread 0 adds the totals.
//
// The slots: a batched record's phantom and handler thread use a slot from the
// lane's free stack from its wake to its end on the chain, and the chain's
// interleaving of those allocations can leave the stack's top entries in
// another order.  The batch allocates nothing and leaves the stack as it is:
// the same set of free slots (every batched thread has ended), so capacity
// failures -- live threads against max_slots -- come out the same, and slot
// numbers are not observable: a ref (tid << 32 | slot) is an opaque handle
// whose thread is named by its tid (the oracle's refs carry no slot at all,
// ref_of in oracle/timedt_oracle.cpp; include/timewarp.h).
#define TW_BATCH_CAP 1024u    // records per lane and window (the rest stay on the chain)
#define TW_BATCH_INSNS 512u   // program tables staged in LDS
#define TW_BATCH_CONSTS 128u
#define TW_BATCH_LPC 256u
// threads per workgroup: two waves, so four workgroups (40.7 KB of LDS each)
// share a CU at the kernel's two waves per SIMD -- a heavy lane's pass is a
// chain of round trips and barriers, and twice the lanes in flight halve the
// rounds (four waves per workgroup: two per CU)
#ifndef TW_BAT_T
#define TW_BAT_T 128u
#endif
#define TW_BAT_RPT (TW_BATCH_CAP / TW_BAT_T)  // records per thread in the prefix scan
static_assert(TW_BAT_T % 64 == 0 && TW_BAT_T <= 256 && TW_BATCH_CAP % TW_BAT_T == 0, "batch workgroup shape");
__global__ void __launch_bounds__(TW_BAT_T) tw_lp_batch(Dev c) {
    const int64_t GAS* w = gp(c.win);
    const int64_t fl = w[WN_FLAGS];
    if (!(fl & WN_FRESH) || (fl & WN_DONE) || !c.lpc_bat) return;
    if (c.n_insns > TW_BATCH_INSNS || c.n_consts > TW_BATCH_CONSTS || c.n_sets * c.n_kinds > TW_BATCH_LPC) return;
    const uint32_t wid = (uint32_t)w[WN_WID];
    const int64_t T0 = w[WN_T], L = w[WN_L];
    const uint32_t lst = wid & 1u;
    uint32_t nh = gp(c.heavy_n)[lst];
    nh = nh < c.R ? nh : c.R;
    if (blockIdx.x >= nh) return;
    __shared__ uint2 sP[TW_BATCH_INSNS];
    __shared__ int64_t sK[TW_BATCH_CONSTS];
    __shared__ uint32_t sL[TW_BATCH_LPC];
    __shared__ uint8_t sB[TW_BATCH_LPC];
    __shared__ uint4 ea[TW_BATCH_CAP + 1], eb[TW_BATCH_CAP];
    __shared__ uint8_t dix[TW_BATCH_CAP];      // per record: batchable | yielded << 1
    __shared__ int64_t wmx[4], sNear[8];
    __shared__ uint64_t sS[SC_COUNT];          // the lane's scalar block
    __shared__ uint32_t bSet, bK0, bK, bDirect, bNd, bNx;
    __shared__ int64_t bTo, bFarT;
    __shared__ uint32_t bSpn;
    __shared__ unsigned long long bH, bsum[6];
    __shared__ long long bFin, bLast;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    for (uint32_t i = tid; i < c.n_insns; i += TW_BAT_T) sP[i] = gp(c.insns)[i];
    for (uint32_t i = tid; i < c.n_consts; i += TW_BAT_T) sK[i] = gp(c.consts)[i];
    for (uint32_t i = tid; i < c.n_sets * c.n_kinds; i += TW_BAT_T) {
        sL[i] = gp(c.lpc)[i];
        sB[i] = gp(c.lpc_bat)[i];
    }
    const BProg bp{(const uint2 LAS*)sP, (const int64_t LAS*)sK, (const uint32_t LAS*)sL, (const uint8_t LAS*)sB};
    const size_t st = ib_stride(c, true);  // (heavy lanes only)
#ifdef TW_STATS
    uint64_t bp_cyc[6] = {0, 0, 0, 0, 0, 0};
#define BT(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#else
#define BT(v) ((void)0)
#endif
    for (uint32_t hi = blockIdx.x; hi < nh; hi += gridDim.x) {
        const uint32_t r = gp(c.heavy)[(size_t)lst * c.R + hi];
        const int64_t T = c.rw ? *rw_at(c, RW_T, r) : T0;
        if (T == INT64_MAX) continue;  // (uniform over the workgroup)
        const int64_t tend = T + L - 1;
        const uint64_t GAS* sc = gp(c.scal) + (size_t)r * SC_LP_STRIDE;
        __syncthreads();  // (the previous lane's readers of the shared words are done)
        BT(bt0);
        // (one round of independent loads: the scalar block, the binding, the
        // lane's near spill and far-heap top -- the lane's next queued event --
        // and its spawn count, whether or not they turn out to be needed)
        if (tid < SC_COUNT) sS[tid] = sc[tid];
        if (tid >= 64u && tid < 64u + TW_NEAR_LP) sNear[tid - 64u] = ent_t(gp(c.near_spill)[(size_t)(tid - 64u) * c.R + r]);
        if (tid == 64u + TW_NEAR_LP) bFarT = c.Q ? ent_t(gp(c.far)[r]) : INT64_MAX;
        if (tid == 65u + TW_NEAR_LP) bSpn = c.lpb ? gp(c.spawn_n)[r] : 0u;
        if (tid == 0) {
            const uint32_t own = gp(c.bind_own)[r], rel = gp(c.bind_rel)[r], bd = gp(c.bind)[r];
            bSet = own == rel ? 0u : bd;
            bK = 0;
            bDirect = 0;
            bH = 0;
            bFin = INT64_MIN;
            bLast = INT64_MIN;
            for (int j = 0; j < 6; ++j) bsum[j] = 0;
        }
        __syncthreads();
        if (tid == 0) {
            const uint32_t nd0 = sS[SC_DUE_H] == 0 ? (uint32_t)sS[SC_DUE_N] : 0u;  // (tw_lp_due's fresh run)
            // a free slot: on the chain each record's phantom takes one at its
            // wake (due_pop -> alloc_slot) and its handler keeps it (DELIVER's
            // in-place fork_); a batched prefix never overlaps two records, so
            // one free slot is what the chain needs -- a full lane stays on the
            // chain, which fails it with TW_REP_ERR_SLOTS at the first due pop
            const bool el = nd0 && c.trace_cap == 0 && c.tie_mode == TW_TIE_FIFO &&
                            (sS[SC_FREE_N] > 0 || sS[SC_BUMP] < (uint64_t)c.S) &&
                            sS[SC_STATUS] == TW_REP_RUNNING && sS[SC_PENDING_MAIN] == 0 &&
                            !bSpn && sS[SC_SEQ] + 3ull * nd0 < 0xFFFFFFFFull &&
                            sS[SC_TIDC] + nd0 < 0xFFFFFFFFull;
            bNx = nd0;  // the due run's length (records past the cap stay on the chain)
            bNd = el ? (nd0 < TW_BATCH_CAP ? nd0 : TW_BATCH_CAP) : 0u;
            bK0 = bNd;
            int64_t to = INT64_MAX;  // the lane's next queued event
            for (uint32_t j = 0; j < TW_NEAR_LP; ++j)
                if (j < (uint32_t)sS[SC_NEAR_N]) to = sNear[j] < to ? sNear[j] : to;
            if (sS[SC_FAR_N]) to = bFarT < to ? bFarT : to;
            bTo = to;
        }
        __syncthreads();
        const uint32_t nd = bNd;
        if (!nd) continue;  // (uniform)
        // the records
        const size_t ib = ib_base(c, r);
        const uint32_t nx = bNx > nd ? nd + 1u : nd;  // (+ the first record past the cap: its time)
        for (uint32_t i = tid; i < nx; i += TW_BAT_T) {
            const uint4 GAS* q = gp(c.due) + (ib + (size_t)i * st) * 2;
            ea[i] = q[0];
            if (i < nd) eb[i] = q[1];
        }
        __syncthreads();
        BT(bt1);
        // dry run: batchable | yielded << 1 per record (due order); each thread
        // keeps its first record's outcome for the effects
        DueX x0{};
        for (uint32_t i = tid; i < nd; i += TW_BAT_T) {
            const DueX x = due_exec(c, bp, r, bSet, ea[i], eb[i]);
            const bool ok = x.ok && x.last < bTo;
            dix[i] = (uint8_t)((ok ? 1u : 0u) | (x.yld ? 2u : 0u));
            if (!ok) atomicMin(&bK0, i);
            if (i == tid) x0 = x;
        }
        __syncthreads();
        BT(bt2);
        const uint32_t K0 = bK0;
        // the latest resume before each position: TW_BAT_RPT records per
        // thread (1,024), an inclusive max scan of the thread maxima (wave
        // shuffles, then the waves)
        {
            int64_t cm = INT64_MIN;
            for (uint32_t j = 0; j < TW_BAT_RPT; ++j) {
                const uint32_t i = tid * TW_BAT_RPT + j;
                if (i < K0 && (dix[i] & 2u)) {
                    const int64_t y = ent_t(ea[i]) + 1;
                    cm = y > cm ? y : cm;
                }
            }
#pragma unroll
            for (uint32_t d = 1; d < 64; d <<= 1) {
                const int64_t o = __shfl_up(cm, d, 64);
                if (lane >= d) cm = o > cm ? o : cm;
            }
            if (lane == 63) wmx[wv] = cm;
            __syncthreads();
            int64_t m = __shfl_up(cm, 1, 64);  // (exclusive within the wave)
            if (lane == 0) m = INT64_MIN;
            for (uint32_t k = 0; k < wv; ++k) m = wmx[k] > m ? wmx[k] : m;
            // (the last thread also checks position TW_BATCH_CAP: a due run of
            // exactly the cap, or the first record past it, may close the prefix)
            const uint32_t jn = tid == TW_BAT_T - 1u ? TW_BAT_RPT + 1u : TW_BAT_RPT;
            for (uint32_t j = 0; j < jn; ++j) {
                const uint32_t i = tid * TW_BAT_RPT + j;
                if (i > K0) break;
                // the prefix [0, i) is kept when its last resume precedes record i's
                // wake (i = nd: the first record past the cap, or none)
                if (i == nd && bNx == nd) { atomicMax(&bK, i); break; }
                const int64_t ti = ent_t(ea[i]);
                if (m < ti) atomicMax(&bK, i);  // (i = 0 always)
                if (i < K0 && (dix[i] & 2u)) m = ti + 1 > m ? ti + 1 : m;
            }
        }
        __syncthreads();
        BT(bt3);
        BT(bt4);
        // the prefix for real: other nodes' hash terms, the sends' records
        const uint32_t K = bK;
        if (!K) continue;  // (uniform)
        {
            const uint32_t node = (c.lp0 + r) >> c.rep_lg;
            uint64_t h = 0;
            uint32_t sm[6] = {0, 0, 0, 0, 0, 0}, dir = 0;
            int64_t fin = INT64_MIN, last = INT64_MIN;
            for (uint32_t i = tid; i < K; i += TW_BAT_T) {
                const DueX x = i == tid ? x0 : due_exec(c, bp, r, bSet, ea[i], eb[i]);
                dir |= due_effects(c, wid, node, x);
                h += x.h;
                sm[0] += x.dl; sm[1] += x.ud; sm[2] += x.dr; sm[3] += x.ev; sm[4] += x.th; sm[5] += x.sq;
                fin = x.fin > fin ? x.fin : fin;
                last = x.last > last ? x.last : last;
            }
            if (h) atomicAdd(&bH, (unsigned long long)h);
            for (int j = 0; j < 6; ++j)
                if (sm[j]) atomicAdd(&bsum[j], (unsigned long long)sm[j]);
            if (dir) bDirect = 1;
            if (fin != INT64_MIN) atomicMax(&bFin, (long long)fin);
            if (last != INT64_MIN) atomicMax(&bLast, (long long)last);
        }
        __syncthreads();
        BT(bt5);
        if (tid == 0) {
            uint64_t GAS* sw = gp(c.scal) + (size_t)r * SC_LP_STRIDE;
            sw[SC_SEQ] = sS[SC_SEQ] + bsum[5];  // (after the due run's reserved seqs)
            sw[SC_DUE_H] = K;
            if (c.bat_ctr) atomicAdd(gp(c.bat_ctr), (unsigned long long)K);
            // the prefix's totals, as its events on the chain add them
            sw[SC_DELIVERED] = sS[SC_DELIVERED] + bsum[0];
            sw[SC_UNDELIV] = sS[SC_UNDELIV] + bsum[1];
            sw[SC_DROPPED] = sS[SC_DROPPED] + bsum[2];
            sw[SC_EVENTS] = sS[SC_EVENTS] + bsum[3];
            sw[SC_THREADS] = sS[SC_THREADS] + bsum[4];
            sw[SC_TIDC] = sS[SC_TIDC] + bsum[0];  // (a thread id per handler)
            if ((int64_t)sS[SC_NOW] < (int64_t)bLast) sw[SC_NOW] = (uint64_t)bLast;
            if ((int64_t)sS[SC_FINAL_T] < (int64_t)bFin) sw[SC_FINAL_T] = (uint64_t)bFin;
            if (bH)
                __hip_atomic_fetch_add((unsigned long long GAS*)(gp(c.hash_g) + c.lp0 + r), bH, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            if (bDirect)  // sent records straight into inboxes (Lane::emit, the event kernel's epilogue)
                min_hot(c.rw ? (uint64_t GAS*)rw_at(c, RW_WIN, r) : (uint64_t GAS*)(gp(c.win) + WN_REC_MIN),
                        (uint64_t)(tend + 1));
        }
#ifdef TW_STATS
        BT(bt6);
        bp_cyc[0] += bt1 - bt0; bp_cyc[1] += bt2 - bt1; bp_cyc[2] += bt3 - bt2;
        bp_cyc[3] += bt4 - bt3; bp_cyc[4] += bt5 - bt4; bp_cyc[5] += bt6 - bt5;
#endif
    }
#ifdef TW_STATS
    if (tid == 0 && c.prof)
        for (int j = 0; j < 6; ++j)
            __hip_atomic_fetch_add(gp(c.prof) + 2 * P_COUNT + j, (unsigned long long)bp_cyc[j], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
#endif
#undef BT
}

// ---------------------------------------------------------------------------
// tw_lp_due + tw_lp_batch in one pass over a heavy lane's records (round 6,
// DESIGN §3i; TW_LP_FUSED=1 -- measured slower than the two kernels, so not
// the default).  A heavy lane's inbox is staged in LDS once: the records
// due in the window are sorted into the due run as tw_lp_due sorts them
// (timestamp bins, then rec_less inside a bin), their reply links looked up
// once, and the batch's dry run, prefix and effects (tw_lp_batch) run on the
// sorted records in LDS -- no second read of the due run, no second launch,
// and only the records the batch leaves (positions [K, nd)) are written back
// as the due run.  The one ordering the two kernels kept: the window's work
// list (tw_lpb_compact) is built from the marks of the window before, and a
// batched reply delivered straight into a light lane's inbox marks that lane
// for the window after -- made now, before the list is built, the mark would
// hide the one the list reads.  So those lanes are recorded (Dev::dmk, by
// window parity) and marked by tw_lp_dmark right after the list is built.
// Everything else is tw_lp_due's and tw_lp_batch's code path for path: the
// reserved seqs of the due run, the records left for later windows and their
// minimum, the heavy list of the next window, the batch's eligibility and
// totals.
__global__ void __launch_bounds__(256) tw_lp_due_batch(Dev c) {
    const int64_t GAS* w = gp(c.win);
    const int64_t fl = w[WN_FLAGS];
    if (!(fl & WN_FRESH) || (fl & WN_DONE)) return;
    const uint32_t wid = (uint32_t)w[WN_WID];
    const int64_t T0 = w[WN_T], L = w[WN_L];
    const bool radix = L <= TW_DUE_BINS;
    const uint32_t nb = radix ? (uint32_t)L : 0u;
    const uint32_t lst = wid & 1u;
    uint32_t nh = gp(c.heavy_n)[lst];
    nh = nh < c.R ? nh : c.R;  // (an over-full list has set lp_err)
    if (blockIdx.x >= nh) return;
    // the batch needs the program tables in LDS (a program over the caps is
    // only sorted, as tw_lp_due alone would)
    const bool tables = c.lpc_bat && c.n_insns <= TW_BATCH_INSNS && c.n_consts <= TW_BATCH_CONSTS &&
                        c.n_sets * c.n_kinds <= TW_BATCH_LPC;
    __shared__ uint4 ea[TW_HEAVY_CAP], eb[TW_HEAVY_CAP];
    __shared__ uint16_t dix[TW_HEAVY_CAP];  // entry index of the i-th due record (arrival order); then batch flags
    __shared__ uint16_t srt[TW_HEAVY_CAP];  // ... of the i-th due record in due-run order
    __shared__ uint32_t bins[TW_DUE_BINS];
    __shared__ uint32_t wsum[4];
    __shared__ unsigned long long smin;
    __shared__ uint2 sP[TW_BATCH_INSNS];
    __shared__ int64_t sK[TW_BATCH_CONSTS];
    __shared__ uint32_t sL[TW_BATCH_LPC];
    __shared__ uint8_t sB[TW_BATCH_LPC];
    __shared__ int64_t wmx[4], sNear[8];
    __shared__ uint64_t sS[SC_COUNT];
    __shared__ uint32_t bSet, bK0, bK, bDirect, bNd;
    __shared__ int64_t bTo;
    __shared__ unsigned long long bH, bsum[6];
    __shared__ long long bFin, bLast;
    static_assert(TW_HEAVY_CAP == 256 * 8, "eight entries per thread");
    static_assert(TW_DUE_BINS == 256 * 8, "eight bins per thread");
    static_assert(TW_BATCH_CAP == 256 * 4, "four prefix positions per thread");
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    if (tables) {
        for (uint32_t i = tid; i < c.n_insns; i += 256) sP[i] = gp(c.insns)[i];
        for (uint32_t i = tid; i < c.n_consts; i += 256) sK[i] = gp(c.consts)[i];
        for (uint32_t i = tid; i < c.n_sets * c.n_kinds; i += 256) {
            sL[i] = gp(c.lpc)[i];
            sB[i] = gp(c.lpc_bat)[i];
        }
    }
    const BProg bp{(const uint2 LAS*)sP, (const int64_t LAS*)sK, (const uint32_t LAS*)sL, (const uint8_t LAS*)sB};
    uint8_t* bfl = (uint8_t*)dix;  // (batch flags per due position, once dix is consumed)
    const size_t st = ib_stride(c, true);  // (heavy lanes only)
    for (uint32_t hi = blockIdx.x; hi < nh; hi += gridDim.x) {
        const uint32_t r = gp(c.heavy)[(size_t)lst * c.R + hi];
        const int64_t T = c.rw ? *rw_at(c, RW_T, r) : T0;
        if (T == INT64_MAX) continue;  // (a finished replica has no records; uniform)
        const int64_t tend = T + L - 1;
        uint64_t* sc = gp(c.scal) + (size_t)r * SC_LP_STRIDE;  // (LP: the lane's block)
        __syncthreads();  // (the previous lane's readers of the shared words are done)
        uint32_t n = gp(c.inbox_n)[r];
        const uint32_t cap = ib_cap(c, r);
        n = n < cap ? n : cap;
        const size_t ib = ib_base(c, r);
        for (uint32_t k = tid; k < n; k += 256) {
            const uint4 GAS* q = gp(c.inbox) + (ib + (size_t)k * st) * 2;
            ea[k] = q[0];
            eb[k] = q[1];
        }
        if (tid < SC_COUNT) sS[tid] = sc[tid];
        if (tid == 0) {
            smin = ~0ull;
            const uint32_t own = gp(c.bind_own)[r], rel = gp(c.bind_rel)[r];
            bSet = own == rel ? 0u : gp(c.bind)[r];
            bK = 0;
            bDirect = 0;
            bH = 0;
            bFin = INT64_MIN;
            bLast = INT64_MIN;
            for (int j = 0; j < 6; ++j) bsum[j] = 0;
        }
        if (tid < 8u) {  // the lane's next queued event: its near spill and far heap top
            int64_t x = INT64_MAX;
            if (tid < (uint32_t)sc[SC_NEAR_N]) x = ent_t(gp(c.near_spill)[(size_t)tid * c.R + r]);
            if (tid == 0 && sc[SC_FAR_N]) {
                const int64_t f = ent_t(gp(c.far)[r]);
                x = f < x ? f : x;
            }
            sNear[tid] = x;
        }
        for (uint32_t i = tid; i < nb; i += 256) bins[i] = 0;
        __syncthreads();
        // ---- tw_lp_due: due flags, a scan, the due records' arrival indices
        // and timestamp bins, the rest compacted back into the inbox
        uint32_t my = 0;
        for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t k = tid * 8 + j;
            my += (k < n && ent_t(ea[k]) <= tend) ? 1u : 0u;
        }
        uint32_t nd = 0;
        uint32_t before = wg_excl_scan(my, wsum, &nd);
        unsigned long long mn = ~0ull;
        for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t k = tid * 8 + j;
            if (k >= n) break;
            const int64_t t = ent_t(ea[k]);
            if (t <= tend) {
                dix[before++] = (uint16_t)k;
                if (radix) atomicAdd(&bins[t > T ? (uint32_t)(t - T) : 0u], 1u);
            } else {
                uint4 GAS* q = gp(c.inbox) + (ib + (size_t)(k - before) * st) * 2;
                q[0] = ea[k];
                q[1] = eb[k];
                mn = (unsigned long long)t < mn ? (unsigned long long)t : mn;
            }
        }
        if (mn != ~0ull) atomicMin(&smin, mn);
        __syncthreads();
        if (radix) {
            uint32_t cnt8[8], sum = 0;
            for (uint32_t j = 0; j < 8; ++j) {
                const uint32_t bi = tid * 8 + j;
                cnt8[j] = bi < nb ? bins[bi] : 0u;
                sum += cnt8[j];
            }
            uint32_t tot = 0;
            uint32_t off = wg_excl_scan(sum, wsum, &tot);
            for (uint32_t j = 0; j < 8; ++j) {
                const uint32_t bi = tid * 8 + j;
                if (bi < nb) bins[bi] = off;
                off += cnt8[j];
            }
            __syncthreads();
            for (uint32_t i = tid; i < nd; i += 256) {
                const uint32_t k = dix[i];
                const int64_t t = ent_t(ea[k]);
                const uint32_t pos = atomicAdd(&bins[t > T ? (uint32_t)(t - T) : 0u], 1u);
                srt[pos] = (uint16_t)k;
            }
            __syncthreads();
            for (uint32_t bi = tid; bi < nb; bi += 256) {
                const uint32_t s0 = bi ? bins[bi - 1] : 0u, s1 = bins[bi];
                for (uint32_t x = s0 + 1; x < s1; ++x) {
                    const uint16_t k = srt[x];
                    uint32_t y = x;
                    while (y > s0 && rec_less(ea[k], eb[k], ea[srt[y - 1]], eb[srt[y - 1]])) {
                        srt[y] = srt[y - 1];
                        --y;
                    }
                    srt[y] = k;
                }
            }
        } else {
            // long windows: rank of every due record among the due ones (ties by arrival)
            for (uint32_t i = tid; i < nd; i += 256) {
                const uint32_t k = dix[i];
                const uint4 a = ea[k], b = eb[k];
                uint32_t rank = 0;
                for (uint32_t j = 0; j < nd; ++j) {
                    const uint32_t m = dix[j];
                    rank += (rec_less(ea[m], eb[m], a, b) || (j < i && !rec_less(a, b, ea[m], eb[m]))) ? 1u : 0u;
                }
                srt[rank] = (uint16_t)k;
            }
        }
        __syncthreads();
        // the due-run format of each due record: its reply link in place of the destination
        for (uint32_t i = tid; i < nd; i += 256) {
            const uint32_t k = srt[i];
            eb[k] = due_rec_b(c, eb[k]);
        }
        // ---- tw_lp_batch's eligibility (the due run is fresh: seqs reserved below)
        const uint64_t s0 = sS[SC_SEQ];
        const bool ctr_ok = s0 + nd < 0xFFFFFFFFull;
        if (tid == 0) {
            const uint64_t sq = s0 + nd;  // (SC_SEQ after the due run's reservation)
            const bool el = tables && nd && ctr_ok && c.trace_cap == 0 && c.tie_mode == TW_TIE_FIFO &&
                            (sS[SC_FREE_N] > 0 || sS[SC_BUMP] < (uint64_t)c.S) &&
                            sS[SC_STATUS] == TW_REP_RUNNING && sS[SC_PENDING_MAIN] == 0 &&
                            !(c.lpb && gp(c.spawn_n)[r]) && sq + 3ull * nd < 0xFFFFFFFFull &&
                            sS[SC_TIDC] + nd < 0xFFFFFFFFull;
            bNd = el ? (nd < TW_BATCH_CAP ? nd : TW_BATCH_CAP) : 0u;
            bK0 = bNd;
            int64_t to = INT64_MAX;
            for (int j = 0; j < 8; ++j) to = sNear[j] < to ? sNear[j] : to;
            bTo = to;
        }
        __syncthreads();
        const uint32_t nbt = bNd;  // (uniform)
        uint32_t K = 0;
        DueX x0{};
        if (nbt) {
            // dry run: batchable | yielded << 1 per record (due order)
            for (uint32_t i = tid; i < nbt; i += 256) {
                const uint32_t k = srt[i];
                const DueX x = due_exec(c, bp, r, bSet, ea[k], eb[k]);
                const bool ok = x.ok && x.last < bTo;
                bfl[i] = (uint8_t)((ok ? 1u : 0u) | (x.yld ? 2u : 0u));
                if (!ok) atomicMin(&bK0, i);
                if (i == tid) x0 = x;
            }
            __syncthreads();
            const uint32_t K0 = bK0;
            // the latest resume before each position (an inclusive max scan)
            int64_t cm = INT64_MIN;
            for (uint32_t j = 0; j < 4; ++j) {
                const uint32_t i = tid * 4 + j;
                if (i < K0 && (bfl[i] & 2u)) {
                    const int64_t y = ent_t(ea[srt[i]]) + 1;
                    cm = y > cm ? y : cm;
                }
            }
#pragma unroll
            for (uint32_t d = 1; d < 64; d <<= 1) {
                const int64_t o = __shfl_up(cm, d, 64);
                if (lane >= d) cm = o > cm ? o : cm;
            }
            if (lane == 63) wmx[wv] = cm;
            __syncthreads();
            int64_t m = __shfl_up(cm, 1, 64);
            if (lane == 0) m = INT64_MIN;
            for (uint32_t k = 0; k < wv; ++k) m = wmx[k] > m ? wmx[k] : m;
            // (the last thread also checks position TW_BATCH_CAP: the first record
            // past the cap may close the prefix)
            const uint32_t jn = tid == 255u ? 5u : 4u;
            for (uint32_t j = 0; j < jn; ++j) {
                const uint32_t i = tid * 4 + j;
                if (i > K0) break;
                // the prefix [0, i) is kept when its last resume precedes record
                // i's wake (i = nbt: the first record past the cap, or none)
                if (i == nbt && nd == nbt) { atomicMax(&bK, i); break; }
                const int64_t ti = ent_t(ea[srt[i]]);
                if (m < ti) atomicMax(&bK, i);
                if (i < K0 && (bfl[i] & 2u)) m = ti + 1 > m ? ti + 1 : m;
            }
            __syncthreads();
            K = bK;
        }
        // ---- the due run the chain pops: positions [K, nd) (the batch took [0, K))
        for (uint32_t i = K + tid; i < nd; i += 256) {
            const uint32_t k = srt[i];
            uint4 GAS* q = gp(c.due) + (ib + (size_t)i * st) * 2;
            q[0] = ea[k];
            q[1] = eb[k];
        }
        // ---- the prefix for real: other nodes' hash terms, the sends' records
        if (K) {
            const uint32_t node = (c.lp0 + r) >> c.rep_lg;
            uint64_t h = 0;
            uint32_t sm[6] = {0, 0, 0, 0, 0, 0}, dir = 0;
            int64_t fin = INT64_MIN, last = INT64_MIN;
            for (uint32_t i = tid; i < K; i += 256) {
                const uint32_t k = srt[i];
                const DueX x = i == tid ? x0 : due_exec(c, bp, r, bSet, ea[k], eb[k]);
                dir |= due_effects(c, wid, node, x, true);
                h += x.h;
                sm[0] += x.dl; sm[1] += x.ud; sm[2] += x.dr; sm[3] += x.ev; sm[4] += x.th; sm[5] += x.sq;
                fin = x.fin > fin ? x.fin : fin;
                last = x.last > last ? x.last : last;
            }
            if (h) atomicAdd(&bH, (unsigned long long)h);
            for (int j = 0; j < 6; ++j)
                if (sm[j]) atomicAdd(&bsum[j], (unsigned long long)sm[j]);
            if (dir) bDirect = 1;
            if (fin != INT64_MIN) atomicMax(&bFin, (long long)fin);
            if (last != INT64_MIN) atomicMax(&bLast, (long long)last);
        }
        __syncthreads();
        if (tid == 0) {
            // tw_lp_due's bookkeeping
            const uint32_t left = n - nd;
            gp(c.inbox_n)[r] = left;
            if (!ctr_ok) {
                if (sS[SC_STATUS] == TW_REP_RUNNING) sc[SC_STATUS] = TW_REP_ERR_COUNTER;
            } else {
                sc[SC_SEQ] = s0 + nd + bsum[5];  // the due run's seqs s0 + 1 .. s0 + nd, then the batch's
            }
            sc[SC_DUE_SEQ] = s0;
            sc[SC_DUE_N] = nd;
            sc[SC_DUE_H] = K;
            if (c.bat_ctr) {
                atomicAdd(gp(c.bat_ctr) + 1, (unsigned long long)nd);
                if (K) atomicAdd(gp(c.bat_ctr), (unsigned long long)K);
            }
            if (smin != ~0ull)
                __hip_atomic_fetch_min(c.rw ? (uint64_t GAS*)rw_at(c, RW_WIN, r) : gp(c.pend_min), (uint64_t)smin,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (nd) lp_mark(c, r, wid - 1u);
            if (left) {
                const uint32_t l = lst ^ 1u;
                const uint32_t i = __hip_atomic_fetch_add(gp(c.heavy_n) + l, 1u, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
                if (i < c.R) gp(c.heavy)[(size_t)l * c.R + i] = r;
                else __hip_atomic_fetch_or(gp(c.lp_err), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            // tw_lp_batch's totals, as the prefix's events on the chain add them
            if (K) {
                sc[SC_DELIVERED] = sS[SC_DELIVERED] + bsum[0];
                sc[SC_UNDELIV] = sS[SC_UNDELIV] + bsum[1];
                sc[SC_DROPPED] = sS[SC_DROPPED] + bsum[2];
                sc[SC_EVENTS] = sS[SC_EVENTS] + bsum[3];
                sc[SC_THREADS] = sS[SC_THREADS] + bsum[4];
                sc[SC_TIDC] = sS[SC_TIDC] + bsum[0];  // (a thread id per handler)
                if ((int64_t)sS[SC_NOW] < (int64_t)bLast) sc[SC_NOW] = (uint64_t)bLast;
                if ((int64_t)sS[SC_FINAL_T] < (int64_t)bFin) sc[SC_FINAL_T] = (uint64_t)bFin;
                if (bH)
                    __hip_atomic_fetch_add((unsigned long long GAS*)(gp(c.hash_g) + c.lp0 + r), bH, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                if (bDirect)
                    min_hot(c.rw ? (uint64_t GAS*)rw_at(c, RW_WIN, r) : (uint64_t GAS*)(gp(c.win) + WN_REC_MIN),
                            (uint64_t)(tend + 1));
            }
        }
    }
}
// The light lanes tw_lp_due_batch delivered batched replies to, marked for the
// next window now that this window's list is built; the other parity's list
// (the window before's, already marked) is emptied for the next window.
__global__ void __launch_bounds__(256) tw_lp_dmark(Dev c) {
    const int64_t GAS* w = gp(c.win);
    const int64_t fl = w[WN_FLAGS];
    if (!(fl & WN_FRESH) || (fl & WN_DONE)) return;
    const uint32_t wid = (uint32_t)w[WN_WID], p = wid & 1u;
    uint32_t n = gp(c.dmk_n)[p];
    n = n < c.dmk_cap ? n : c.dmk_cap;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
        lp_mark(c, gp(c.dmk)[(size_t)p * c.dmk_cap + i], wid);
    if (blockIdx.x == 0 && threadIdx.x == 0) gp(c.dmk_n)[p ^ 1u] = 0;
}

// Batched LP: a replica's results = its nodes' lanes (lane = node << rep_lg |
// replica) reduced on the device: counts summed, final time the latest, status
// the worst error (else done), the main exception whichever lane holds one.
// out: [8][n_rep] words (final_t, events, delivered, dropped, undeliverable,
// status, main_exc, threads).
// Batched LP: per-replica results over the replica's node lanes.  A wave
// reads 64 replicas' words of one node (coalesced); the nodes are split over
// the grid's y dimension and the four waves of a workgroup, the partials
// combined in LDS and then by atomics into `out` (zeroed by the caller):
// sums for the counters, max for final_t and the worst status (floored at
// TW_REP_DONE), and for main_exc the last node with one -- (node + 1) << 32 |
// code, its max -- as the serial loop over nodes chose.
#define TW_RED_GROUPS 64  // node groups: grid.y x 4 waves
__global__ void __launch_bounds__(256) tw_lpb_reduce(Dev c, uint64_t* out) {
    const uint32_t nr = 1u << c.rep_lg;
    const uint32_t q = blockIdx.x * 64 + (threadIdx.x & 63u);
    const uint32_t g = blockIdx.y * 4 + (threadIdx.x >> 6);
    const uint32_t per = (c.Ntot + TW_RED_GROUPS - 1) / TW_RED_GROUPS;
    const uint32_t n0 = g * per, n1 = n0 + per < c.Ntot ? n0 + per : c.Ntot;
    int64_t ft = 0;
    uint64_t ev = 0, dl = 0, dr = 0, ud = 0, th = 0, me = 0, st = TW_REP_DONE;
    if (q < nr) {
        for (uint32_t n = n0; n < n1; ++n) {
            const uint64_t GAS* sc = gp(c.scal) + ((((size_t)n << c.rep_lg) + q) * SC_LP_STRIDE);
            const int64_t f = (int64_t)sc[SC_FINAL_T];
            ft = f > ft ? f : ft;
            ev += sc[SC_EVENTS]; dl += sc[SC_DELIVERED]; dr += sc[SC_DROPPED];
            ud += sc[SC_UNDELIV]; th += sc[SC_THREADS];
            const uint64_t x = sc[SC_MAIN_EXC], s2 = sc[SC_STATUS];
            me = x ? ((uint64_t)(n + 1) << 32) | (x & 0xFFFFFFFFull) : me;
            st = (s2 >= TW_REP_ABORTED && s2 > st) ? s2 : st;
        }
    }
    __shared__ uint64_t part[8][4][64];
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63u;
    part[0][w][l] = (uint64_t)ft; part[1][w][l] = ev; part[2][w][l] = dl; part[3][w][l] = dr;
    part[4][w][l] = ud; part[5][w][l] = st; part[6][w][l] = me; part[7][w][l] = th;
    __syncthreads();
    if (threadIdx.x < 64 && q < nr) {
        for (int k = 1; k < 4; ++k) {
            ft = (int64_t)part[0][k][l] > ft ? (int64_t)part[0][k][l] : ft;
            ev += part[1][k][l]; dl += part[2][k][l]; dr += part[3][k][l]; ud += part[4][k][l];
            st = part[5][k][l] > st ? part[5][k][l] : st;
            me = part[6][k][l] > me ? part[6][k][l] : me;
            th += part[7][k][l];
        }
        uint64_t GAS* o = gp(out);
        auto add = [&](int f, uint64_t v) {
            if (v) __hip_atomic_fetch_add((unsigned long long GAS*)(o + (size_t)f * nr + q), (unsigned long long)v,
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        };
        auto mx = [&](int f, uint64_t v) {
            __hip_atomic_fetch_max((unsigned long long GAS*)(o + (size_t)f * nr + q), (unsigned long long)v,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        };
        mx(0, (uint64_t)(ft > 0 ? ft : 0));  // (final times are >= 0)
        add(1, ev); add(2, dl); add(3, dr); add(4, ud);
        mx(5, st);
        mx(6, me);
        add(7, th);
    }
}

// tw_run's statistics on the device, instead of copying every replica's
// results to the host (248 MB for C2's million replicas): out[0] the events
// of this run (the events word minus its value at the run's start), [1..3]
// delivered / dropped / undeliverable, [4] the largest final time, [5] / [6]
// replicas done / in an error status.  A wave reduces its 64 replicas, its
// first lane adds them in with atomics (out zeroed by the caller).
__device__ __forceinline__ unsigned long long shx64(unsigned long long v, int m) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, 64);
    return ((unsigned long long)hi << 32) | lo;
}
__global__ void __launch_bounds__(256) tw_stats_kernel(Dev c, const uint64_t* ev0, unsigned long long* out) {
    const size_t r = (size_t)blockIdx.x * 256 + threadIdx.x;
    unsigned long long v[7] = {0ull, 0ull, 0ull, 0ull, 0ull, 0ull, 0ull};
    if (r < c.R) {
        const uint64_t GAS* s = gp(c.scal);
        v[0] = s[sc_ix(c, SC_EVENTS, r)] - gp(ev0)[r];
        v[1] = s[sc_ix(c, SC_DELIVERED, r)];
        v[2] = s[sc_ix(c, SC_DROPPED, r)];
        v[3] = s[sc_ix(c, SC_UNDELIV, r)];
        const int64_t ft = (int64_t)s[sc_ix(c, SC_FINAL_T, r)];
        v[4] = ft > 0 ? (unsigned long long)ft : 0ull;
        const uint32_t st = (uint32_t)s[sc_ix(c, SC_STATUS, r)];
        v[5] = st == TW_REP_DONE ? 1ull : 0ull;
        v[6] = st >= TW_REP_ERR_SLOTS ? 1ull : 0ull;
    }
#pragma unroll
    for (int k = 0; k < 7; ++k) {
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            const unsigned long long o = shx64(v[k], m);
            v[k] = k == 4 ? (o > v[k] ? o : v[k]) : v[k] + o;
        }
    }
    if (__lane_id() == 0) {
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            if (k == 4)
                __hip_atomic_fetch_max(gp(out) + k, v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else if (v[k])
                __hip_atomic_fetch_add(gp(out) + k, v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Per-replica digest of the results and node hashes (tw_tie_audit compares
// runs under different tie orders without copying every hash to the host).
__global__ void __launch_bounds__(256) tw_digest_kernel(Dev c, uint64_t* out) {
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= c.R) return;
    uint64_t d = 0;
    const int fields[8] = {SC_FINAL_T, SC_EVENTS, SC_DELIVERED, SC_DROPPED, SC_UNDELIV, SC_STATUS, SC_MAIN_EXC,
                           SC_THREADS};
    for (int i = 0; i < 8; ++i) d = mix64(d ^ gp(c.scal)[sc_ix(c, fields[i], r)]) + (uint64_t)i;
    for (uint32_t n = 0; n < c.N; ++n) d += mix64(gp(c.hash)[(size_t)n * c.R + r] ^ ((uint64_t)n * 0x9e3779b97f4a7c15ull));
    gp(out)[r] = d;
}


}  // namespace
