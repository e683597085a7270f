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
//     FIFO runs and a 4-ary heap in HBM for far events; the record the next
//     pop most likely needs is loaded into LDS staging by LDS-DMA one step
//     ahead, so the common pop -> run -> re-queue cycle rarely waits on HBM;
//   * every thread has at most one queued event, so throwTo's queue rebuild
//     (TimedT.hs:361-368) becomes an O(1) re-stamp: a fresh (now, seq) entry is
//     pushed (or the near entry re-keyed in place) and a superseded entry is
//     dropped lazily at pop time (slot.wake_seq no longer matches);
//   * the event order is (t, seq) with seq a per-replica insertion counter —
//     bit-identical to the oracle's canonical mode.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/timewarp.h"
#include "tw_dev.hpp"
#include "shard.hpp"

#include "engine_dev.hpp"

// ======================================================================= C ABI
struct tw_shard {
    int device = 0;
    hipStream_t stream = nullptr;
    Dev d{};
    bool loaded = false;
    std::vector<void*> allocs;
    uint32_t* h_active = nullptr;  // pinned
    // tw_run's statistics reduced on the device (tw_stats_kernel): the events
    // column at the run's start, the 8 result words, their pinned host copy
    uint64_t* st_ev0 = nullptr;
    unsigned long long* st_out = nullptr;
    unsigned long long* h_st = nullptr;
    uint32_t main_pc = 0, main_node = 0;
    int64_t* main_regs = nullptr;  // device copies for tw_reset
    int64_t* nv_init = nullptr;
    uint32_t* listen_init = nullptr;
    size_t lds_bytes = 0;
    int geo = 0;  // 0: dense (TW_WG, TW_NEAR_CAP); 1: sparse (TW_WG_SPARSE, TW_NEAR_SPARSE); 2: half (TW_WG, TW_NEAR_CAP, TW_HALF_LANES lanes per wave)
    // LP mode
    bool lp = false;
    bool lpb = false;               // batched LP (tw_lpb_load): R = nodes x replicas
    uint32_t n_rep = 1;             // replicas batched per node
    bool heavy_ok = false;          // some node's inbox can exceed TW_LIGHT (tw_lp_due runs)
    uint64_t lpb_windows = 0, lpb_ticks = 0;  // of the last batched-LP tw_run
    bool lpb_fresh = false;         // tw_reset since the last batched-LP tw_run: every counter is 0
    bool has_ph1 = false;           // two-phase windows (Dev::phase)
    uint4* foreign = nullptr;      // [out_cap][2]
    uint32_t* n_foreign = nullptr;
    uint4* staging = nullptr;      // inject staging [out_cap][2]
    std::vector<double> launch_ms;
    std::vector<hipEvent_t> ev_pool;
    std::vector<uint32_t> tie_flags;  // tw_tie_audit, per replica
    Dev* d_dev = nullptr;             // device copy of d (the wave kernel reads it through the scalar cache)
    uint32_t seq0 = 0, tid0 = 1;      // tw_set_counter_base
    hipStream_t own_stream = nullptr; // the context's stream (tw_set_stream may replace `stream`)
    // device-driven windows (tw_lp_exchange_setup / sh_lp_exchange_own):
    // blocks of ex_cap records (the stride) of which the first ex_cap_eff go
    // over the wire this tick (<= ex_cap; the library loop adapts it)
    uint32_t ex_world = 1, ex_rank = 0, ex_cap = 0, ex_cap_eff = 0;
    uint32_t* ex_starts = nullptr;    // device, world + 1
    uint4* ex_send = nullptr;         // caller's device buffers (or ex_own's)
    uint4* ex_recv = nullptr;
    int64_t* ex_red = nullptr;        // caller's (or red_own, or ex_own's)
    int64_t* red_own = nullptr;
    void* ex_own = nullptr;           // library-owned send | recv | red (sh_lp_exchange_own)
    void* ex_carry = nullptr;         // Dev::carry + carry_n
    int64_t* win_buf = nullptr;       // the device loop's WN_* words
    int64_t* h_win = nullptr;         // pinned host copy of them + lp_err (tw_lp_progress)
    bool loop_ready = false;
    // sh_lp_run_windows: TW_GRAPH_TICKS ticks + the progress copy captured as
    // one hipGraph (a tick is 4-8 short kernels: launched one by one, the host's
    // enqueue rate left the device idle between them), re-captured when the
    // launch arguments it holds change (tick_gkey)
    hipGraphExec_t tick_graph = nullptr;
    std::vector<unsigned char> tick_gkey;
    // pops per lane per tick of the device loop (TW_LP_TICK_BUDGET overrides it,
    // for tests: a small budget makes windows take several ticks)
    uint32_t lp_budget = 1u << 14;
    uint32_t lp_grid = TW_LP_GRID;  // LP launches above this many workgroups walk the list (TW_LP_GRID env)
    Dev dwin() const {                // the descriptor the device loop's kernels get
        Dev x = d;
        x.win = win_buf;
        return x;
    }
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
int dalloc(tw_shard* c, T** p, size_t n) {
    void* q = nullptr;
    if (n == 0) n = 1;
    HIPCHK(hipMalloc(&q, n * sizeof(T)));
    c->allocs.push_back(q);
    *p = (T*)q;
    return TW_OK;
}

void free_all(tw_shard* c) {
    for (void* p : c->allocs) (void)hipFree(p);
    c->allocs.clear();
    if (c->d.trace) (void)hipFree(c->d.trace);
    c->d.trace = nullptr;
    c->d.trace_cap = 0;
    if (c->ex_starts) (void)hipFree(c->ex_starts);
    if (c->ex_own) (void)hipFree(c->ex_own);
    if (c->ex_carry) (void)hipFree(c->ex_carry);
    c->ex_starts = nullptr;
    c->ex_own = c->ex_carry = nullptr;
    c->d.carry = nullptr;
    c->d.carry_n = nullptr;
    c->d.carry_cap = 0;
    c->ex_send = c->ex_recv = nullptr;
    c->ex_red = c->red_own = nullptr;
    c->win_buf = nullptr;
    c->ex_world = 1;
    c->ex_rank = c->ex_cap = c->ex_cap_eff = 0;
    c->loop_ready = false;
    if (c->st_ev0) (void)hipFree(c->st_ev0);
    if (c->st_out) (void)hipFree(c->st_out);
    c->st_ev0 = nullptr;
    c->st_out = nullptr;
    if (c->tick_graph) (void)hipGraphExecDestroy(c->tick_graph);
    c->tick_graph = nullptr;
    c->tick_gkey.clear();
    c->loaded = false;
}

}  // namespace

// The fork-in-place variant (Lane::fork_in_place) of a replica geometry: under
// the tie orders where a forked child is always the next pop (FORKFIRST,
// LIFO), and for the compact geometry in every order.  Measured (round 4):
// C3 dense FIFO 17.8 G events/s without it, 16.3 G with it (the child is
// rarely next under FIFO and the code costs registers), FORKFIRST 19.4 G;
// C2 compact FIFO 39.7 G without, 43.2-44.0 G with (ping-pong forks into an
// empty queue: the child is next under FIFO too)
static bool use_ip(const tw_shard* c) {
    if (c->lp || c->geo == 1) return false;  // (LP: its own inline paths; sparse: compiled out)
    return c->d.tie_mode == TW_TIE_FORKFIRST || c->d.tie_mode == TW_TIE_LIFO || c->geo == 7;
}

template <bool LP, int WG, int NC, int TPW = 64, bool RUNS = true>
static void launch_run(tw_shard* c, hipStream_t st, int64_t t_end, uint64_t limit, uint32_t budget) {
    const uint32_t blocks = (uint32_t)((c->d.R + WG - 1) / WG);
    const bool ip = !LP && WG >= 64 && use_ip(c);
    if constexpr (LP) {
        // many lanes, few listed: the work list walked grid-stride (GS); the
        // batched device loop's per-replica windows (PRW)
        const bool gs = blocks > c->lp_grid, prw = c->d.rw && c->d.win;
        const dim3 g(gs ? c->lp_grid : blocks), b(WG * 64 / TPW);
        if (gs && prw)
            hipLaunchKernelGGL((tw_run_kernel<LP, WG, NC, TPW, RUNS, true, true>), g, b, c->lds_bytes, st, c->d, t_end,
                               limit, budget);
        else if (gs)
            hipLaunchKernelGGL((tw_run_kernel<LP, WG, NC, TPW, RUNS, true, false>), g, b, c->lds_bytes, st, c->d, t_end,
                               limit, budget);
        else if (prw)
            hipLaunchKernelGGL((tw_run_kernel<LP, WG, NC, TPW, RUNS, false, true>), g, b, c->lds_bytes, st, c->d, t_end,
                               limit, budget);
        else
            hipLaunchKernelGGL((tw_run_kernel<LP, WG, NC, TPW, RUNS>), g, b, c->lds_bytes, st, c->d, t_end, limit,
                               budget);
    } else {
        if constexpr (WG >= 64) {
            if (ip) {
                hipLaunchKernelGGL((tw_run_kernel<LP, WG, NC, TPW, RUNS, false, false, true>), dim3(blocks),
                                   dim3(WG * 64 / TPW), c->lds_bytes, st, c->d, t_end, limit, budget);
                return;
            }
        }
        hipLaunchKernelGGL((tw_run_kernel<LP, WG, NC, TPW, RUNS>), dim3(blocks), dim3(WG * 64 / TPW), c->lds_bytes, st,
                           c->d, t_end, limit, budget);
    }
}

namespace tw {

int sh_create(int device, tw_shard** out) {
    if (!out) return TW_ERR_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device < 0 || device >= n) return TW_ERR_NO_DEVICE;
    {
        // the kernels are built for gfx950 (MI355X) only
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) != hipSuccess || strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            return TW_ERR_NO_DEVICE;
    }
    tw_shard* c = new (std::nothrow) tw_shard;
    if (!c) return TW_ERR_OOM;
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc((void**)&c->h_active, sizeof(uint32_t)) != hipSuccess) {
        delete c;
        return TW_ERR_HIP;
    }
    c->own_stream = c->stream;
    *out = c;
    return TW_OK;
}

void sh_destroy(tw_shard* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    free_all(c);
    for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
    if (c->h_active) (void)hipHostFree(c->h_active);
    if (c->h_st) (void)hipHostFree(c->h_st);
    if (c->h_win) (void)hipHostFree(c->h_win);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
}

static int validate(const tw_scenario_desc* s) {
    if (!s || s->abi_version != TW_ABI_VERSION) return TW_ERR_INVALID;
    if (s->n_replicas == 0 || s->n_nodes == 0 || !s->insns || s->n_insns < TW_PC_USER || s->n_insns > 0xFFFF)
        return TW_ERR_INVALID;
    if (s->max_slots < 1 || s->queue_capacity < 1 || s->link_depth < 1 || !s->out_off) return TW_ERR_INVALID;
    if (s->max_frames > TW_MAX_FRAMES) return TW_ERR_INVALID;
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

int sh_reset(tw_shard* c);

// Batch class of every resume pc for the wave kernel (wave.hip PC_*): what the
// code a thread runs from that pc until its next yield may touch.
//   1 (LOCAL)   its own record, its own node's vars / binding / out-links, and
//               forks (whose records and queue entries the batch commit writes);
//   2 (DELIVER) LOCAL plus the destination node of a delivery (the deliverer stub);
//   0 (ALONE)   anything that can reach another thread or another node's state
//               (throwTo, throw, the watchdog's fire, cross-node vars, in-place
//               handlers): such an event runs as a batch of one.
// Events in one batch have equal timestamps, consecutive seqs and disjoint node
// footprints, so running them side by side commits the same effects as
// TimedT's one-at-a-time loop (TimedT.hs:239-263).  (Sends go over the sender's
// own out-links, as every lowered scenario's LINK / RLINK links do.)
static void classify_pcs(const tw_scenario_desc* s, std::vector<uint8_t>& cls) {
    const uint32_t n = s->n_insns;
    cls.assign((size_t)n + 1, 0);
    bool inline_any = false;
    for (size_t i = 0; i < (size_t)s->n_listener_sets * s->n_msg_kinds; ++i)
        if (s->listener_pc[i] != TW_PC_NONE && (s->listener_pc[i] & TW_LPC_INLINE)) inline_any = true;
    std::vector<uint32_t> seen(n, 0xFFFFFFFFu), stk;
    for (uint32_t p0 = 0; p0 < n; ++p0) {
        bool alone = false, dlv = false;
        stk.assign(1, p0);
        seen[p0] = p0;
        while (!stk.empty() && !alone) {
            const uint32_t q = stk.back();
            stk.pop_back();
            const uint32_t op = s->insns[q].w0 & 0xFFu;
            const uint32_t imm = (uint32_t)s->insns[q].imm;
            uint32_t nx[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};
            switch (op) {
            case TW_OP_THROW_TO: case TW_OP_THROW: case TW_OP_TMO_FIRE: case TW_OP_NLOADX: case TW_OP_NSTOREX:
                alone = true;
                break;
            case TW_OP_END: case TW_OP_WAIT_REL: case TW_OP_WAIT_ABS: case TW_OP_WAIT_REG: case TW_OP_FORK:
            case TW_OP_TMO_BEGIN:
                break;  // the step ends here
            case TW_OP_DELIVER:
                if (inline_any) alone = true;
                dlv = true;
                nx[0] = q + 1;  // undeliverable: the deliverer goes on
                break;
            case TW_OP_JMP:
                nx[0] = imm;
                break;
            case TW_OP_JEQ: case TW_OP_JNE: case TW_OP_JLT: case TW_OP_JLE: case TW_OP_JEQI: case TW_OP_JNEI:
                nx[0] = imm;
                nx[1] = q + 1;
                break;
            default:
                if (op >= TW_OP_COUNT) alone = true;
                nx[0] = q + 1;  // (SEND: a dropped message lets the sender go on)
                break;
            }
            for (uint32_t x : nx) {
                if (x == 0xFFFFFFFFu) continue;
                if (x >= n) { alone = true; break; }
                if (seen[x] != p0) { seen[x] = p0; stk.push_back(x); }
            }
        }
        cls[p0] = alone ? 0 : dlv ? 2 : 1;
    }
}

// The handlers a heavy lane's due run may execute data-parallel (tw_lp_due,
// round 5): the fork_-dispatched handler of a (listener set, kind) whose code,
// on every path from its entry, touches only its own registers, reads its
// node's variables, computes out-links and reply links, traces, and sends at
// most once with END right after the send -- bench/Network's Ping handler
// `reply Pong` (Receiver/Main.hs:32-38; ForkStrategy fork_, MonadDialog.hs:317).
// Such a handler's effects are its own (hash terms, counters, one record), so
// records whose events no other event of the lane interleaves with can run one
// per thread with the totals of the sequential loop.  Forward jumps only (the
// walk is bounded by the image); no NSTORE, fork, wait, throw, listen or MYTID.
static void classify_batch(const tw_scenario_desc* s, std::vector<uint8_t>& bat) {
    const uint32_t n = s->n_insns, nk = s->n_msg_kinds;
    bat.assign((size_t)s->n_listener_sets * nk, 0);
    auto op_at = [&](uint32_t q) { return q < n ? s->insns[q].w0 & 0xFFu : 0xFFu; };
    std::vector<uint32_t> seen(n, 0xFFFFFFFFu), stk;
    for (size_t e = 0; e < bat.size(); ++e) {
        const uint32_t lpc = s->listener_pc[e];
        if (lpc == TW_PC_NONE || (lpc & TW_LPC_INLINE) || lpc >= n) continue;
        bool ok = true;
        stk.assign(1, lpc);
        seen[lpc] = (uint32_t)e;
        while (!stk.empty() && ok) {
            const uint32_t q = stk.back();
            stk.pop_back();
            const uint32_t w = s->insns[q].w0, op = w & 0xFFu, b = w >> 16;
            const uint32_t imm = (uint32_t)s->insns[q].imm;
            uint32_t nx[2] = {q + 1, 0xFFFFFFFFu};
            switch (op) {
            case TW_OP_END: nx[0] = 0xFFFFFFFFu; break;
            case TW_OP_NOP: case TW_OP_MOV: case TW_OP_ADD: case TW_OP_SUB: case TW_OP_NLOAD: case TW_OP_LINK:
            case TW_OP_RLINK:
                break;
            case TW_OP_SETI: case TW_OP_SETK: case TW_OP_ADDI: case TW_OP_MULI: case TW_OP_NOW: case TW_OP_NODE:
                ok = !(b & TW_ALU_NSTORE);  // (the fused NSTORE writes a node variable)
                break;
            case TW_OP_TRACE:
                if (b & TW_TRACE_PAIR) nx[0] = q + 2;
                break;
            case TW_OP_JMP: case TW_OP_JEQ: case TW_OP_JNE: case TW_OP_JLT: case TW_OP_JLE: case TW_OP_JEQI:
            case TW_OP_JNEI:
                ok = imm > q && imm < n;
                nx[0] = imm;
                nx[1] = op == TW_OP_JMP ? 0xFFFFFFFFu : q + 1;
                break;
            case TW_OP_SEND: {
                // the send yields 1 µs (it forks the deliverer): the thread must end there
                const uint32_t k = (b & (TW_SEND_VIA_LINK | TW_SEND_VIA_RLINK)) ? q + 2 : q + 1;
                ok = op_at(k) == TW_OP_END;
                nx[0] = 0xFFFFFFFFu;
                break;
            }
            default: ok = false; break;
            }
            for (uint32_t x : nx) {
                if (x == 0xFFFFFFFFu || !ok) continue;
                if (x >= n) { ok = false; break; }
                if (seen[x] != (uint32_t)e) { seen[x] = (uint32_t)e; stk.push_back(x); }
            }
        }
        bat[e] = ok ? 1 : 0;
    }
}

static int load_common(tw_shard* c, const tw_scenario_desc* s, bool lp, uint32_t lp_begin, uint32_t lp_count,
                       int64_t lookahead, uint32_t inbox_cap, uint32_t outbox_cap, bool lpb = false,
                       const uint32_t* node_caps = nullptr) {
    if (!c) return TW_ERR_INVALID;
    int v = validate(s);
    if (v) return v;
    uint32_t rep_lg = 0;
    if (lpb) {
        // every replica's nodes as lanes (node-major): a power-of-two replica count
        while ((1u << rep_lg) < s->n_replicas) ++rep_lg;
        if ((1u << rep_lg) != s->n_replicas || rep_lg > 16 || (uint64_t)s->n_nodes << rep_lg > 0x7FFFFFFFull ||
            outbox_cap < 2 || lookahead < 1)
            return TW_ERR_INVALID;
        uint64_t tot = 0;
        for (uint32_t n = 0; n < s->n_nodes; ++n) {
            const uint32_t k = node_caps ? node_caps[n] : inbox_cap;
            if (k == 0 || k > TW_HEAVY_CAP) return TW_ERR_INVALID;
            tot += k;
        }
        if ((tot << rep_lg) > 0x7FFFFFFFull) return TW_ERR_INVALID;  // (a lane's inbox base: 31 bits, DW_IB)
        lp_begin = 0;
        lp_count = s->n_nodes << rep_lg;
    } else if (lp && (s->n_replicas != 1 || lp_count == 0 || (uint64_t)lp_begin + lp_count > s->n_nodes ||
                      inbox_cap == 0 || inbox_cap > TW_LIGHT || outbox_cap == 0 || lookahead < 1)) {
        return TW_ERR_INVALID;
    }
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    free_all(c);
    Dev& d = c->d;
    d = Dev{};
    c->lp = lp;
    c->lpb = lpb;
    c->n_rep = lpb ? s->n_replicas : 1u;
    c->heavy_ok = false;
    c->has_ph1 = false;
    d.rep_lg = rep_lg;
    d.lpb = lpb ? 1u : 0u;
    d.R = lp ? lp_count : s->n_replicas;
    d.S = s->max_slots; d.Q = s->queue_capacity;
    d.RQ = lp ? 1u : (uint64_t)d.S * d.R;  // quad stride: LP records contiguous (Lane::hrec)
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
    if (lp) d.Cr = 0;  // LP nodes keep no far runs (tw_run_kernel<true> has no LDS for them)
    d.max_frames = s->max_frames ? s->max_frames : 2u;
    d.FXQ = d.max_frames > 2 ? (d.max_frames - 2 + 3) / 4 : 0u;
    d.tie_mode = TW_TIE_FIFO;
    c->tie_flags.assign(d.R, 0u);
    const size_t R = d.R;
    const size_t Rt = s->n_replicas;  // replica dimension of the host tables
    const size_t prog_lds = 16ull * (d.n_insns + 1) + 8ull * d.n_consts + 4ull * d.n_sets * d.n_kinds;
    // geometry by replica count (TW_GEOMETRY overrides; LP mode is dense):
    // <= 4096: a wavefront per replica (C5: 0.32 G events/s vs 0.25 sparse,
    // 0.20 narrow); < 65536: narrow (C3 at 8192: 2.5 vs 0.99 sparse, 0.74
    // wave); else dense (one workgroup of 256 per CU)
    {
        const char* g = getenv("TW_GEOMETRY");
        // dense batches of a scenario without far runs (run_capacity 0, e.g.
        // C2's ping-pong: every event within the near horizon) take the
        // compact geometry: two waves per SIMD
        int geo = lp ? 0 : R <= 4096 ? 3 : R < 65536 ? 5 : (s->run_capacity == 0 ? 7 : 0);
        if (g && !strcmp(g, "dense")) geo = 0;
        if (g && !strcmp(g, "compact")) geo = 7;
        if (g && !strcmp(g, "sparse")) geo = 1;
        if (g && !strcmp(g, "half")) geo = 2;
        if (g && !strcmp(g, "wave")) geo = 3;
        if (g && !strcmp(g, "narrow")) geo = 5;
        if (lp) geo = 0;
        if (geo == 1 && fixed_lds_bytes<TW_WG_SPARSE, TW_NEAR_SPARSE>() + prog_lds > 160 * 1024) geo = 0;
        c->geo = geo;
    }
    if (c->geo == 7) d.Cr = 0;  // far events: the HBM heap only
    c->lds_bytes = (lp            ? fixed_lds_bytes<TW_WG_LP, TW_NEAR_LP, true>()
                    : c->geo == 7 ? fixed_lds_bytes<TW_WG, TW_NEAR_COMPACT, false, false>()
                    : c->geo == 1 ? fixed_lds_bytes<TW_WG_SPARSE, TW_NEAR_SPARSE>()
                    : c->geo == 5 ? fixed_lds_bytes<TW_NARROW, TW_NEAR_CAP>()
                                  : fixed_lds_bytes<TW_WG, TW_NEAR_CAP>()) +
                   prog_lds;
    if (c->geo == 3) c->lds_bytes = 0;  // the wave kernel reads the program image through the scalar cache
    if (c->lds_bytes > 160 * 1024) { free_all(c); return TW_ERR_INVALID; }  // program + constants must fit in LDS
    {
        // (the kernel and, for the lane-per-replica geometries, its fork-in-place variant)
        auto lds = [&](const void* k) { return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                                    (int)c->lds_bytes); };
        if (c->geo == 3) {
        } else if (lp) {
            HIPCHK(lds((const void*)tw_run_kernel<true, TW_WG_LP, TW_NEAR_LP>));
        } else if (c->geo == 1) {
            HIPCHK(lds((const void*)tw_run_kernel<false, TW_WG_SPARSE, TW_NEAR_SPARSE>));
        } else if (c->geo == 2) {
            HIPCHK(lds((const void*)tw_run_kernel<false, TW_WG, TW_NEAR_CAP, TW_HALF_LANES>));
            HIPCHK(lds((const void*)tw_run_kernel<false, TW_WG, TW_NEAR_CAP, TW_HALF_LANES, true, false, false, true>));
        } else if (c->geo == 5) {
            HIPCHK(lds((const void*)tw_run_kernel<false, TW_NARROW, TW_NEAR_CAP, TW_NARROW>));
            HIPCHK(lds((const void*)tw_run_kernel<false, TW_NARROW, TW_NEAR_CAP, TW_NARROW, true, false, false, true>));
        } else if (c->geo == 7) {
            HIPCHK(lds((const void*)tw_run_kernel<false, TW_WG, TW_NEAR_COMPACT, 64, false>));
            HIPCHK(lds((const void*)tw_run_kernel<false, TW_WG, TW_NEAR_COMPACT, 64, false, false, false, true>));
        } else {
            HIPCHK(lds((const void*)tw_run_kernel<false, TW_WG, TW_NEAR_CAP>));
            HIPCHK(lds((const void*)tw_run_kernel<false, TW_WG, TW_NEAR_CAP, 64, true, false, false, true>));
        }
    }
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
    d.sc_lp = lp ? 1u : 0u;  // LP lanes: one contiguous scalar block per lane (sc_ix)
    ALLOC(d.scal, (size_t)(lp ? SC_LP_STRIDE : SC_COUNT) * R);
    ALLOC(d.slots, (size_t)d.S * R * 4);
    ALLOC(d.free_stk, (size_t)d.S * R);
    ALLOC(d.far, (size_t)d.Q * R);
    ALLOC(d.runs, (size_t)(d.Cr ? TW_RUNS * (size_t)d.Cr : 1) * R);
    if (c->geo == 3) d.wave_k = (uint32_t)wave_near_k(d.R);
    ALLOC(d.near_spill, (size_t)(lp ? TW_NEAR_LP : c->geo == 1 ? TW_NEAR_SPARSE : c->geo == 3 ? wave_spill_entries(d.wave_k) : TW_NEAR_CAP) * R);
    ALLOC(d.dummy, (size_t)TW_DUMMY_REC + R);
    ALLOC(d.nvars, (size_t)d.N * 4 * R);
    ALLOC(d.hash, (size_t)d.N * R);
    ALLOC(d.bind, (size_t)d.N * R);
    ALLOC(d.bind_own, (size_t)d.N * R);
    ALLOC(d.bind_rel, (size_t)d.N * R);
    ALLOC(d.link_ord, (size_t)(d.L ? d.L : 1) * (lp ? (size_t)1 << rep_lg : R));
    ALLOC(d.tmo_done, (size_t)(d.T ? d.T : 1) * R);
    ALLOC(d.n_active, 1);
    ALLOC(c->d_dev, 1);
    if (d.FXQ) ALLOC(d.fx, (size_t)d.S * R * d.FXQ);
    uint32_t* mbytes = nullptr;
    uint64_t* lbw = nullptr;
    if (s->msg_bytes && s->link_bw && d.n_kinds && d.L) {
        ALLOC(mbytes, d.n_kinds);
        ALLOC(lbw, d.L);
    }
#ifdef TW_STATS
    ALLOC(d.prof, 2 * P_COUNT + TW_BPROF);
    HIPCHK(hipMemsetAsync(d.prof, 0, 8 * (2 * P_COUNT + TW_BPROF), c->stream));
#endif
    uint32_t* iboff = nullptr;
    std::vector<uint32_t> h_iboff;
    uint8_t* phd = nullptr;
    std::vector<uint8_t> h_ph;
    if (lpb) {
        // two-phase windows: a link shorter than the lookahead (over every
        // replica and ordinal) must run from a phase-0 node into a node that
        // then runs in phase 1 (after phase 0 has finished the window), and such
        // a node's inbox must be light (drained at phase 1's first tick)
        h_ph.assign(s->n_nodes, 0);
        std::vector<uint8_t> shortl(s->n_links, 0);
        for (uint32_t l = 0; l < s->n_links; ++l) {
            uint32_t dmin = 0;
            if (s->link_table) {
                dmin = 0x7FFFFFFFu;
                const uint32_t* e = s->link_table + (size_t)l * s->link_depth * s->n_replicas;
                for (size_t i = 0; i < (size_t)s->link_depth * s->n_replicas; ++i) {
                    const uint32_t v = e[i] & 0x7FFFFFFFu;
                    dmin = v < dmin ? v : dmin;
                }
            }
            if ((int64_t)dmin < lookahead) {
                shortl[l] = 1;
                h_ph[s->link_dst[l]] = 1;
            }
        }
        for (uint32_t n = 0; n < s->n_nodes; ++n)
            for (uint32_t l = s->out_off[n]; l < s->out_off[n + 1]; ++l)
                if (shortl[l] && h_ph[n]) { free_all(c); return TW_ERR_INVALID; }
        for (uint32_t n = 0; n < s->n_nodes; ++n) {
            if (!h_ph[n]) continue;
            c->has_ph1 = true;
            if ((node_caps ? node_caps[n] : inbox_cap) > TW_LIGHT) { free_all(c); return TW_ERR_INVALID; }
        }
    }
    if (lp) {
        if (c->has_ph1) {
            ALLOC(phd, h_ph.size());
        }
        size_t ib_entries = (size_t)d.IB * R;
        if (lpb) {
            h_iboff.resize((size_t)s->n_nodes + 1);
            h_iboff[0] = 0;
            for (uint32_t n = 0; n < s->n_nodes; ++n) {
                const uint32_t k = node_caps ? node_caps[n] : inbox_cap;
                h_iboff[n + 1] = h_iboff[n] + k;
                if (k > TW_LIGHT) c->heavy_ok = true;
            }
            ib_entries = (size_t)h_iboff[s->n_nodes] << rep_lg;
            d.IB = 0;
            ALLOC(iboff, h_iboff.size());
            ALLOC(d.spawn, (size_t)TW_SPN * R * 4);
            ALLOC(d.spawn_n, R);
        }
        ALLOC(d.hash_g, (size_t)d.Ntot << rep_lg);
        ALLOC(d.inbox, ib_entries * 2 * 2);  // two buffers (Dev::dpar)
        d.ib_total = ib_entries;
        ALLOC(d.due, c->heavy_ok ? ib_entries * 2 : 2);
        ALLOC(d.heavy, c->heavy_ok ? 2 * R : 2);
        ALLOC(d.heavy_n, 2);
        if (lpb) ALLOC(d.bat_ctr, 2);
        // tw_lp_due_batch's deferred marks: at most one per batched reply, and a
        // window's replies fit its outbox
        d.dmk = nullptr;
        d.dmk_n = nullptr;
        d.dmk_cap = 0;
        if (lpb && c->heavy_ok) {
            d.dmk_cap = d.out_cap;
            ALLOC(d.dmk, (size_t)2 * d.dmk_cap);
            ALLOC(d.dmk_n, 2);
        }
        ALLOC(d.pend_min, 1);
        ALLOC(d.inbox_n, 2 * R);
        ALLOC(d.outbox, (size_t)d.out_cap * 2);
        ALLOC(d.out_n, 1);
        ALLOC(d.next_t, 1);
        ALLOC(d.lp_err, 1);
        ALLOC(d.act, 2 * TW_LP_NB * R);
        ALLOC(d.act_n, 2 * TW_LP_NB);
        ALLOC(d.wake, R);
        ALLOC(d.listed, R);
        {
            const size_t nsb = (R + (1u << TW_SUB_LG) - 1) >> TW_SUB_LG;
            ALLOC(d.sb_mark, nsb);
            ALLOC(d.sb_scan, nsb);
            ALLOC(d.sb_min, nsb);
        }
        if (lpb) ALLOC(d.inlist, R);
        // per-replica windows (TW_LPB_GLOBAL=1: one window for the whole batch)
        d.rw = nullptr;
        d.cw_min = nullptr;
        d.cw_mark = nullptr;
        if (lpb && !getenv("TW_LPB_GLOBAL")) {
            ALLOC(d.rw, (size_t)RW_COUNT << rep_lg);
            const size_t nk = ((R >> rep_lg) + (1u << TW_CHUNK_LG) - 1) >> TW_CHUNK_LG;
            ALLOC(d.cw_min, nk << rep_lg);
            ALLOC(d.cw_mark, nk << rep_lg);
        }
        ALLOC(c->foreign, (size_t)d.out_cap * 2);
        ALLOC(c->n_foreign, 1);
        ALLOC(c->staging, (size_t)d.out_cap * 2);
        ALLOC(c->win_buf, WN_COUNT);  // d.win stays null: the host-driven loop
        ALLOC(c->red_own, RD_COUNT);
    }
    int64_t *mregs = nullptr, *nvi = nullptr;
    if (s->main_regs && (!lp || lpb)) ALLOC(mregs, (size_t)s->n_replicas * 4);
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
    if (mregs) HIPCHK(hipMemcpyAsync(mregs, s->main_regs, 32ull * s->n_replicas, hipMemcpyHostToDevice, st));
    if (iboff) HIPCHK(hipMemcpy(iboff, h_iboff.data(), 4 * h_iboff.size(), hipMemcpyHostToDevice));
    d.ib_off = iboff;
    if (phd) HIPCHK(hipMemcpy(phd, h_ph.data(), h_ph.size(), hipMemcpyHostToDevice));
    if (lp) {
        // destination of every link with the heavy bit of its node (a send to a
        // heavy node goes through tw_lp_pack, to a light one straight in)
        std::vector<uint4> h_dh(d.L ? d.L : 1, make_uint4(0, 0, 0, 0));
        for (uint32_t l = 0; l < d.L; ++l) {
            const uint32_t n = s->link_dst[l];
            const uint32_t cap = lpb ? (node_caps ? node_caps[n] : inbox_cap) : d.IB;
            const bool heavy = lpb && cap > TW_LIGHT;
            h_dh[l] = make_uint4(n | (heavy ? 0x80000000u : 0u), lpb ? h_iboff[n] : 0u, cap, 0u);
        }
        uint4* ldh = nullptr;
        if ((e = dalloc(c, &ldh, h_dh.size())) != TW_OK) { free_all(c); return e; }
        HIPCHK(hipMemcpy(ldh, h_dh.data(), 16 * h_dh.size(), hipMemcpyHostToDevice));
        d.link_dsth = ldh;
        d.dpar = c->has_ph1 ? 0u : 1u;  // (phase-1 lanes drain inside the window: one buffer)
    }
    d.phase = phd;
    d.has_ph1 = c->has_ph1 ? 1u : 0u;
    if (nvi) HIPCHK(hipMemcpyAsync(nvi, s->node_vars, 32ull * d.Ntot, hipMemcpyHostToDevice, st));
    if (lsi) HIPCHK(hipMemcpyAsync(lsi, s->node_listen, 4ull * d.Ntot, hipMemcpyHostToDevice, st));
    if (mbytes) {
        HIPCHK(hipMemcpyAsync(mbytes, s->msg_bytes, 4ull * d.n_kinds, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(lbw, s->link_bw, 8ull * d.L, hipMemcpyHostToDevice, st));
    }
    d.msg_bytes = mbytes;
    d.link_bw = lbw;
    if (c->geo == 3) {
        std::vector<uint8_t> cls;
        classify_pcs(s, cls);
        uint8_t* pcl = nullptr;
        if ((e = dalloc(c, &pcl, cls.size())) != TW_OK) { free_all(c); return e; }
        HIPCHK(hipMemcpy(pcl, cls.data(), cls.size(), hipMemcpyHostToDevice));
        d.pc_cls = pcl;
    }
    d.lpc_bat = nullptr;
    if (lpb && !c->has_ph1 && d.D == 1 && d.n_sets && !(getenv("TW_LP_BATCH") && getenv("TW_LP_BATCH")[0] == '0')) {
        std::vector<uint8_t> bat;
        classify_batch(s, bat);
        bool any = false;
        for (uint8_t x : bat) any = any || x;
        if (any) {
            uint8_t* bd = nullptr;
            if ((e = dalloc(c, &bd, bat.size())) != TW_OK) { free_all(c); return e; }
            HIPCHK(hipMemcpy(bd, bat.data(), bat.size(), hipMemcpyHostToDevice));
            d.lpc_bat = bd;
        }
    }
    d.insns = insns; d.consts = consts; d.lpc = lpc; d.out_off = out_off; d.link_dst = ldst; d.link_rev = lrev;
    d.link_table = ltab;
    c->main_pc = s->main_pc;
    c->main_node = s->main_node;
    c->main_regs = mregs;
    c->nv_init = nvi;
    c->listen_init = lsi;
    c->loaded = true;
    int rc = sh_reset(c);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(st));
    return TW_OK;
}

int sh_load(tw_shard* c, const tw_scenario_desc* s) { return load_common(c, s, false, 0, 0, 0, 0, 0); }

int sh_lp_load(tw_shard* c, const tw_scenario_desc* s, uint32_t lp_begin, uint32_t lp_count, int64_t lookahead_us,
               uint32_t inbox_cap, uint32_t outbox_cap) {
    return load_common(c, s, true, lp_begin, lp_count, lookahead_us, inbox_cap, outbox_cap);
}

int sh_lpb_load(tw_shard* c, const tw_scenario_desc* s, int64_t lookahead_us, const uint32_t* node_inbox_cap,
                uint32_t inbox_cap, uint32_t outbox_cap) {
    return load_common(c, s, true, 0, 0, lookahead_us, inbox_cap, outbox_cap, true, node_inbox_cap);
}

int sh_reset(tw_shard* c) {
    if (!c) return TW_ERR_INVALID;
    if (!c->loaded) return TW_ERR_STATE;
    HIPCHK(hipSetDevice(c->device));
    const Dev& d = c->d;
    const size_t R = d.R;
    hipStream_t st = c->stream;
    HIPCHK(hipMemsetAsync(d.nvars, 0, 32ull * d.N * R, st));
    HIPCHK(hipMemsetAsync(d.hash, 0, 8ull * d.N * R, st));
    HIPCHK(hipMemsetAsync(d.bind, 0, 4ull * d.N * R, st));
    HIPCHK(hipMemsetAsync(d.link_ord, 0, 4ull * (d.L ? d.L : 1) * (c->lp ? (size_t)1 << d.rep_lg : R), st));
    HIPCHK(hipMemsetAsync(d.tmo_done, 0, (size_t)(d.T ? d.T : 1) * R, st));
    if (c->lp) {
        HIPCHK(hipMemsetAsync(d.hash_g, 0, 8ull * ((size_t)d.Ntot << d.rep_lg), st));
        HIPCHK(hipMemsetAsync(d.heavy_n, 0, 8, st));
        if (d.bat_ctr) HIPCHK(hipMemsetAsync(d.bat_ctr, 0, 16, st));
        if (d.dmk_n) HIPCHK(hipMemsetAsync(d.dmk_n, 0, 8, st));
        if (d.inlist) HIPCHK(hipMemsetAsync(d.inlist, 0, 4ull * R, st));
        HIPCHK(hipMemsetAsync(d.pend_min, 0xFF, 8, st));
        HIPCHK(hipMemsetAsync(d.out_n, 0, 4, st));
        HIPCHK(hipMemsetAsync(d.lp_err, 0, 4, st));
        HIPCHK(hipMemsetAsync(c->n_foreign, 0, 4, st));
        c->d.act_cur = 0;
        c->d.wid = 0;
        HIPCHK(hipMemsetAsync(d.act_n, 0, 8 * TW_LP_NB, st));
        c->lpb_fresh = c->lpb;
    }
    if (d.pq_hdr) {
        // empty MinQueues: no element, no node used, every rank a Skip
        std::vector<uint32_t> h((size_t)R * PQ_WORDS, 0u);
        for (size_t r = 0; r < R; ++r)
            for (int k = 0; k < 32; ++k) h[r * PQ_WORDS + PQ_FOREST + k] = 0xFFFFFFFFu;
        HIPCHK(hipMemcpyAsync(d.pq_hdr, h.data(), 4 * h.size(), hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));
    }
    uint32_t blocks = (uint32_t)((R + TW_WG - 1) / TW_WG);
    hipLaunchKernelGGL(tw_init_kernel, dim3(blocks), dim3(TW_WG), 0, st, d, c->main_pc, c->main_node,
                       (const int64_t*)c->main_regs, (const int64_t*)c->nv_init, (const uint32_t*)c->listen_init,
                       c->lp ? 1 : 0, c->seq0, c->tid0);
    HIPCHK(hipGetLastError());
    return TW_OK;
}


static int lpb_run(tw_shard* c, tw_stats* out);

int sh_run(tw_shard* c, int64_t t_end_us, uint64_t max_events, tw_stats* out) {
    if (!c) return TW_ERR_INVALID;
    if (!c->loaded) return TW_ERR_STATE;
    if (c->lpb) {
        // the batched window loop runs every replica to quiescence
        if (t_end_us != INT64_MAX || max_events != UINT64_MAX) return TW_ERR_INVALID;
        return lpb_run(c, out);
    }
    auto w0 = std::chrono::steady_clock::now();
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    const Dev& d = c->d;
    // events before this call (to report per-call deltas; only when asked
    // for: an LP window would otherwise copy 8 B per node every window)
    // (a device-side copy of the events column; tw_stats_kernel reduces the
    // run's statistics on the device at the end)
    if (out) {
        if (!c->st_ev0) HIPCHK(hipMalloc((void**)&c->st_ev0, 8ull * (d.R ? d.R : 1)));
        if (!c->st_out) HIPCHK(hipMalloc((void**)&c->st_out, 64));
        if (!c->h_st) HIPCHK(hipHostMalloc((void**)&c->h_st, 64));
        if (d.sc_lp)  // (the events word of every lane's block: one strided copy)
            HIPCHK(hipMemcpy2DAsync(c->st_ev0, 8, d.scal + SC_EVENTS, 8ull * SC_LP_STRIDE, 8, d.R,
                                    hipMemcpyDeviceToDevice, st));
        else
            HIPCHK(hipMemcpyAsync(c->st_ev0, d.scal + (size_t)SC_EVENTS * d.R, 8ull * d.R, hipMemcpyDeviceToDevice,
                                  st));
    }
    const uint64_t limit = max_events;  // cumulative per-replica cap
    c->launch_ms.clear();
    if (c->lp) {
        // a new window: serve the list built since the last call (nodes with a
        // live thread or new records); start an empty one for the next call
        c->d.act_cur ^= 1u;
        HIPCHK(hipMemsetAsync(d.act_n + c->d.act_cur * TW_LP_NB, 0, 4 * TW_LP_NB, st));
        hipLaunchKernelGGL(tw_lp_compact, dim3(compact_blocks(d.R)), dim3(256), 0, st, c->d, c->d.wid, c->d.act_cur);
        HIPCHK(hipGetLastError());
        c->d.wid += 1u;
    }
    // loop iterations (pops) per lane per launch: bounded kernel time
    static const uint32_t budget = [] {
        const char* b = getenv("TW_LAUNCH_BUDGET");
        const long v = b ? strtol(b, nullptr, 10) : 0;
        return v >= 1 && v <= (1L << 24) ? (uint32_t)v : (1u << 14);
    }();
    // launches between host checks: a replica run needs several budgets; an LP
    // window is almost always done after one launch
    const int per_check = c->lp ? 1 : 4;
    uint32_t launches = 0;
    double kms = 0.0;
    bool quiet = false;
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
                launch_run<true, TW_WG_LP, TW_NEAR_LP>(c, st, t_end_us, limit, budget);
            else if (c->geo == 3)
                HIPCHK(wave_launch(c->d, c->d_dev, st, t_end_us, limit, 1u << 16));
            else if (c->geo == 1)
                launch_run<false, TW_WG_SPARSE, TW_NEAR_SPARSE>(c, st, t_end_us, limit, budget);
            else if (c->geo == 2)
                launch_run<false, TW_WG, TW_NEAR_CAP, TW_HALF_LANES>(c, st, t_end_us, limit, budget);
            else if (c->geo == 5)
                launch_run<false, TW_NARROW, TW_NEAR_CAP, TW_NARROW>(c, st, t_end_us, limit, budget);
            else if (c->geo == 7)
                launch_run<false, TW_WG, TW_NEAR_COMPACT, 64, false>(c, st, t_end_us, limit, budget);
            else
                launch_run<false, TW_WG, TW_NEAR_CAP>(c, st, t_end_us, limit, budget);
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
        if (*c->h_active == 0) { quiet = true; break; }
    }
    if (out) {
        std::memset(out, 0, sizeof(*out));
        HIPCHK(hipMemsetAsync(c->st_out, 0, 64, st));
        hipLaunchKernelGGL(tw_stats_kernel, dim3((uint32_t)((d.R + 255) / 256)), dim3(256), 0, st, d,
                           (const uint64_t*)c->st_ev0, c->st_out);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(c->h_st, c->st_out, 64, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        const unsigned long long* h = c->h_st;
        out->events = h[0];
        out->delivered = h[1];
        out->dropped = h[2];
        out->undeliverable = h[3];
        out->max_final_t = (int64_t)h[4];
        out->replicas_done = (uint32_t)h[5];
        out->replicas_error = (uint32_t)h[6];
        out->sends = out->delivered + out->dropped + out->undeliverable;
        out->launches = launches;
        out->kernel_ms = kms;
        out->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
    }
    return quiet ? TW_OK : TW_ERR_INCOMPLETE;
}

int sh_read_results(tw_shard* c, tw_replica_result* out, size_t n) {
    if (!c || !out) return TW_ERR_INVALID;
    if (!c->loaded) return TW_ERR_STATE;
    const Dev& d = c->d;
    if (n < (c->lpb ? c->n_rep : d.R)) return TW_ERR_INVALID;
    HIPCHK(hipSetDevice(c->device));
    if (c->lpb) {
        const uint32_t nr = c->n_rep;
        uint64_t* dd = nullptr;
        HIPCHK(hipMallocAsync((void**)&dd, 64ull * nr, c->stream));
        HIPCHK(hipMemsetAsync(dd, 0, 64ull * nr, c->stream));
        hipLaunchKernelGGL(tw_lpb_reduce, dim3((nr + 63) / 64, TW_RED_GROUPS / 4), dim3(256), 0, c->stream, d, dd);
        HIPCHK(hipGetLastError());
        std::vector<uint64_t> h(8ull * nr);
        HIPCHK(hipMemcpyAsync(h.data(), dd, 64ull * nr, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipFreeAsync(dd, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        for (uint32_t q = 0; q < nr; ++q) {
            tw_replica_result& o = out[q];
            std::memset(&o, 0, sizeof(o));
            o.final_t = (int64_t)h[q]; o.events = h[nr + q]; o.delivered = h[2ull * nr + q];
            o.dropped = h[3ull * nr + q]; o.undeliverable = h[4ull * nr + q]; o.status = (uint32_t)h[5ull * nr + q];
            o.main_exc = (uint32_t)h[6ull * nr + q];  // (the node tag is in the high word)
            o.threads = h[7ull * nr + q];
        }
        return TW_OK;
    }
    const size_t nsc = (size_t)(d.sc_lp ? SC_LP_STRIDE : SC_COUNT) * d.R;
    std::vector<uint64_t> sc(nsc);
    HIPCHK(hipMemcpyAsync(sc.data(), d.scal, 8ull * nsc, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    auto F = [&](int f, uint32_t i) { return d.sc_lp ? sc[(size_t)i * SC_LP_STRIDE + f] : sc[(size_t)f * d.R + i]; };
    for (uint32_t i = 0; i < d.R; ++i) {
        out[i].final_t = (int64_t)F(SC_FINAL_T, i); out[i].events = F(SC_EVENTS, i);
        out[i].delivered = F(SC_DELIVERED, i); out[i].dropped = F(SC_DROPPED, i);
        out[i].undeliverable = F(SC_UNDELIV, i); out[i].status = (uint32_t)F(SC_STATUS, i);
        out[i].main_exc = (uint32_t)F(SC_MAIN_EXC, i); out[i].threads = F(SC_THREADS, i);
        out[i].tie_flags = i < c->tie_flags.size() ? c->tie_flags[i] : 0u;
        out[i].reserved = 0;
    }
    return TW_OK;
}

static int digest(tw_shard* c, std::vector<uint64_t>& h) {
    const Dev& d = c->d;
    uint64_t* dd = nullptr;
    HIPCHK(hipMallocAsync((void**)&dd, 8ull * d.R, c->stream));
    hipLaunchKernelGGL(tw_digest_kernel, dim3((d.R + 255) / 256), dim3(256), 0, c->stream, d, dd);
    HIPCHK(hipGetLastError());
    h.resize(d.R);
    HIPCHK(hipMemcpyAsync(h.data(), dd, 8ull * d.R, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipFreeAsync(dd, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return TW_OK;
}

int sh_tie_audit(tw_shard* c, int64_t t_end_us, uint64_t max_events, uint32_t probes, tw_stats* out) {
    if (!c) return TW_ERR_INVALID;
    if (!c->loaded) return TW_ERR_STATE;
    if (c->lp || probes < 1 || probes > 2) return TW_ERR_INVALID;
    HIPCHK(hipSetDevice(c->device));
    std::vector<std::vector<uint64_t>> dg(probes + 1);
    int rc = TW_OK;
    for (uint32_t p = probes; p + 1 > 0 && rc == TW_OK; --p) {  // probes first, the canonical run last
        c->d.tie_mode = p;
        rc = sh_reset(c);
        if (rc == TW_OK) rc = sh_run(c, t_end_us, max_events, p == 0 ? out : nullptr);
        if (rc == TW_OK) rc = digest(c, dg[p]);
        if (p == 0) break;
    }
    c->d.tie_mode = TW_TIE_FIFO;
    if (rc != TW_OK) return rc;
    c->tie_flags.assign(c->d.R, 1u);
    for (uint32_t p = 1; p <= probes; ++p)
        for (uint32_t i = 0; i < c->d.R; ++i)
            if (dg[p][i] != dg[0][i]) c->tie_flags[i] |= 1u << p;
    return TW_OK;
}

int sh_geometry(tw_shard* c) {
    if (!c) return TW_ERR_INVALID;
    if (!c->loaded) return TW_ERR_STATE;
    return c->lpb ? TW_GEO_LPB : c->lp ? TW_GEO_LP : c->geo;
}

// The equal-timestamp order of later runs (include/timewarp.h tw_set_tie_mode).
// TW_TIE_PQUEUE runs the wave kernel with each replica's queue as pqueue's
// binomial MinQueue (wave.hip); its node links, free stack, rebuild scratch
// and header are allocated here on first use.
int sh_set_tie_mode(tw_shard* c, uint32_t mode) {
    if (!c) return TW_ERR_INVALID;
    if (!c->loaded) return TW_ERR_STATE;
    if (mode > TW_TIE_FORKFIRST) return TW_ERR_INVALID;
    // a forked child first: the lane-per-replica kernels (their fork_in_place);
    // the wave and logical-process kernels keep the other orders
    if (mode == TW_TIE_FORKFIRST && (c->lp || c->geo == 3)) return TW_ERR_INVALID;
    if (mode == TW_TIE_PQUEUE) {
        if (c->lp || c->geo != 3) return TW_ERR_INVALID;  // the wave kernel only
        HIPCHK(hipSetDevice(c->device));
        HIPCHK(hipStreamSynchronize(c->stream));
        Dev& d = c->d;
        const size_t n = (size_t)d.Q * d.R;
        int e;
        if (!d.pq_link) {
            if ((e = dalloc(c, &d.pq_link, n)) != TW_OK) return e;
            if ((e = dalloc(c, &d.pq_free, n)) != TW_OK) return e;
            if ((e = dalloc(c, &d.pq_scr, n)) != TW_OK) return e;
            if ((e = dalloc(c, &d.pq_hdr, (size_t)d.R * PQ_WORDS)) != TW_OK) return e;
        }
    }
    c->d.tie_mode = mode;
    return TW_OK;
}

int sh_set_counter_base(tw_shard* c, uint32_t seq0, uint32_t tid0) {
    if (!c || tid0 == 0) return TW_ERR_INVALID;
    c->seq0 = seq0;
    c->tid0 = tid0;
    return TW_OK;
}

int sh_read_hashes(tw_shard* c, uint64_t* out, size_t n) {
    if (!c || !out) return TW_ERR_INVALID;
    if (!c->loaded) return TW_ERR_STATE;
    const Dev& d = c->d;
    if (n < (size_t)d.R * d.N) return TW_ERR_INVALID;
    HIPCHK(hipSetDevice(c->device));
    if (c->lpb) {  // hash_g is [node][replica] over the batch too
        std::vector<uint64_t> tmp((size_t)d.Ntot << d.rep_lg);
        HIPCHK(hipMemcpyAsync(tmp.data(), d.hash_g, 8 * tmp.size(), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        for (uint32_t node = 0; node < d.Ntot; ++node)
            for (uint32_t q = 0; q < c->n_rep; ++q) out[(size_t)q * d.Ntot + node] = tmp[((size_t)node << d.rep_lg) | q];
        return TW_OK;
    }
    std::vector<uint64_t> tmp((size_t)d.R * d.N);  // device layout [node][replica]
    HIPCHK(hipMemcpyAsync(tmp.data(), d.hash, 8ull * d.R * d.N, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (uint32_t node = 0; node < d.N; ++node)
        for (uint32_t r = 0; r < d.R; ++r) out[(size_t)r * d.N + node] = tmp[(size_t)node * d.R + r];
    return TW_OK;
}

static int lp_scatter(tw_shard* c, const uint4* recs, uint32_t n, bool to_foreign) {
    const Dev& d = c->d;
    if (n == 0) return TW_OK;
    uint32_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(tw_lp_scatter, dim3(blocks), dim3(256), 0, c->stream, d, recs, n,
                       to_foreign ? c->foreign : nullptr, c->n_foreign, d.out_cap);
    HIPCHK(hipGetLastError());
    return TW_OK;
}

int sh_lp_window(tw_shard* c, int64_t t_end_excl, int64_t* next_t, uint64_t* n_foreign) {
    if (!c || !next_t) return TW_ERR_INVALID;
    if (!c->loaded || !c->lp) return TW_ERR_STATE;
    tw_stats st{};
    int rc = sh_run(c, t_end_excl - 1, UINT64_MAX, nullptr);
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

int sh_lp_take_outbox(tw_shard* c, tw_lp_record* out, size_t cap, size_t* n) {
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

int sh_lp_inject(tw_shard* c, const tw_lp_record* recs, size_t n, int64_t* next_t) {
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

int sh_lp_results(tw_shard* c, tw_replica_result* agg, uint64_t* node_hashes, size_t n_nodes) {
    if (!c || !agg) return TW_ERR_INVALID;
    if (!c->loaded || !c->lp) return TW_ERR_STATE;
    const Dev& d = c->d;
    std::vector<tw_replica_result> rr(d.R);
    int rc = sh_read_results(c, rr.data(), rr.size());
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

int sh_set_stream(tw_shard* c, void* hs) {
    if (!c) return TW_ERR_INVALID;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));  // finish what was queued on the old one
    c->stream = hs ? (hipStream_t)hs : c->own_stream;
    return TW_OK;
}

// The exchange of the device loop over `world` ranks; this shard is `rank`,
// owning nodes [starts[rank], starts[rank + 1]).  send/recv: world blocks of
// (cap + 1) records (header + records); red: RD_COUNT int64.  Also sizes the
// carry buffer (records beyond a tick's block size wait there).
static int exchange_common(tw_shard* c, uint32_t world, uint32_t rank, const uint32_t* starts, uint32_t cap) {
    if (!c || world == 0 || rank >= world || !starts) return TW_ERR_INVALID;
    if (!c->loaded || !c->lp) return TW_ERR_STATE;
    if (world > 1 && cap == 0) return TW_ERR_INVALID;
    for (uint32_t g = 0; g < world; ++g)
        if (starts[g] > starts[g + 1]) return TW_ERR_INVALID;
    if (starts[rank] != c->d.lp0 || starts[rank + 1] != c->d.lp0 + c->d.R) return TW_ERR_INVALID;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (c->ex_starts) HIPCHK(hipFree(c->ex_starts));
    if (c->ex_carry) HIPCHK(hipFree(c->ex_carry));
    c->ex_starts = nullptr;
    c->ex_carry = nullptr;
    c->d.carry = nullptr;
    c->d.carry_n = nullptr;
    c->d.carry_cap = 0;
    HIPCHK(hipMalloc((void**)&c->ex_starts, 4ull * (world + 1)));
    HIPCHK(hipMemcpy(c->ex_starts, starts, 4ull * (world + 1), hipMemcpyHostToDevice));
    if (world > 1) {
        // a tick's foreign records beyond the block size: at most a tick's outbox
        const uint32_t cc = c->d.out_cap < (1u << 20) ? c->d.out_cap : (1u << 20);
        const size_t bytes = 2ull * cc * 32 + 256;
        HIPCHK(hipMalloc(&c->ex_carry, bytes));
        HIPCHK(hipMemsetAsync(c->ex_carry, 0, bytes, c->stream));
        c->d.carry_n = (uint32_t*)c->ex_carry;
        c->d.carry = (uint4*)((char*)c->ex_carry + 256);
        c->d.carry_cap = cc;
    }
    c->ex_world = world;
    c->ex_rank = rank;
    c->ex_cap = cap;
    c->ex_cap_eff = c->ex_cap;
    return TW_OK;
}

int sh_lp_exchange_setup(tw_shard* c, uint32_t world, uint32_t rank, const uint32_t* starts, void* send, void* recv,
                         uint32_t cap, int64_t* red) {
    if (c && world > 1 && (!send || !recv || !red)) return TW_ERR_INVALID;
    int rc = exchange_common(c, world, rank, starts, cap);
    if (rc) return rc;
    if (c->ex_own) HIPCHK(hipFree(c->ex_own));
    c->ex_own = nullptr;
    c->ex_send = world > 1 ? (uint4*)send : nullptr;
    c->ex_recv = world > 1 ? (uint4*)recv : nullptr;
    c->ex_red = world > 1 ? red : c->red_own;
    if (world > 1) HIPCHK(hipMemsetAsync(send, 0, 32ull * world * (cap + 1), c->stream));
    return TW_OK;
}

// The same with library-owned buffers (the library-driven loop of abi.hip:
// RCCL send/recv or device copies between shards move the blocks).
int sh_lp_exchange_own(tw_shard* c, uint32_t world, uint32_t rank, const uint32_t* starts, uint32_t cap) {
    int rc = exchange_common(c, world, rank, starts, world > 1 ? cap : 1u);
    if (rc) return rc;
    if (c->ex_own) HIPCHK(hipFree(c->ex_own));
    c->ex_own = nullptr;
    const size_t blk = 32ull * world * ((size_t)c->ex_cap + 1);
    HIPCHK(hipMalloc(&c->ex_own, 2 * blk + 8ull * RD_COUNT));
    HIPCHK(hipMemsetAsync(c->ex_own, 0, 2 * blk + 8ull * RD_COUNT, c->stream));
    // (one rank too: its import, fill and the all-reduce of the words then go
    // through the transport -- a one-rank RCCL communicator -- like any rank's)
    c->ex_send = (uint4*)c->ex_own;
    c->ex_recv = (uint4*)((char*)c->ex_own + blk);
    c->ex_red = (int64_t*)((char*)c->ex_own + 2 * blk);
    return TW_OK;
}

void sh_lp_exchange_info(tw_shard* c, ShardXchg* x) {
    x->device = c->device;
    x->stream = c->stream;
    x->send = c->ex_send;
    x->recv = c->ex_recv;
    x->red = c->ex_red;
    x->world = c->ex_world;
    x->stride = c->ex_cap;
    x->cap_eff = c->ex_cap_eff;
}
int sh_lp_set_block(tw_shard* c, uint32_t cap_eff) {
    if (!c || cap_eff == 0 || cap_eff > c->ex_cap) return TW_ERR_INVALID;
    c->ex_cap_eff = cap_eff;
    return TW_OK;
}
// WN_XMAX after a tw_lp_progress (the largest per-rank demand of one tick since
// the last clear); clear it on the device (stream-ordered)
int64_t sh_lp_xmax(tw_shard* c) { return c->h_win ? c->h_win[WN_XMAX] : 0; }
int sh_lp_clear_xmax(tw_shard* c) {
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemsetAsync(c->win_buf + WN_XMAX, 0, 8, c->stream));
    return TW_OK;
}


// A fresh window's start (every tick launches it; the kernels return unless
// the window is fresh): the heavy lanes' due runs (tw_lp_due), the work list
// from the last window's marks (tw_lpb_compact / tw_lp_compact), then the
// due runs' batchable prefixes (tw_lp_batch: its replies' marks are the next
// window's, so after the list).  Where the batch runs, tw_lp_due_batch does
// both in one pass over each heavy lane's records (round 6) and tw_lp_dmark
// makes its marks after the list -- measured slower (C5 1,463 -> 1,708 ms per
// step: one 89-KB workgroup per CU runs the batch's dry runs that the separate
// tw_lp_batch runs three workgroups per CU wide), so only with
// TW_LP_FUSED=1 (A/B).
static int lp_window_start(tw_shard* c) {
    static const bool fused = getenv("TW_LP_FUSED") && getenv("TW_LP_FUSED")[0] == '1';
    const bool bat = c->heavy_ok && c->d.lpc_bat;
    const bool fuse = bat && fused && c->d.dmk;
    if (c->heavy_ok) {
        if (fuse) hipLaunchKernelGGL(tw_lp_due_batch, dim3(TW_DUE_GRID), dim3(256), 0, c->stream, c->dwin());
        else hipLaunchKernelGGL(tw_lp_due, dim3(TW_DUE_GRID), dim3(256), 0, c->stream, c->dwin());
        HIPCHK(hipGetLastError());
    }
    if (c->d.rw) {  // per-replica windows: tiles of 64 replicas x one chunk of nodes, four per workgroup
        const uint32_t nk = ((c->d.R >> c->d.rep_lg) + (1u << TW_CHUNK_LG) - 1u) >> TW_CHUNK_LG;
        const uint32_t tiles = nk * (((1u << c->d.rep_lg) + 63u) >> 6);
        hipLaunchKernelGGL(tw_lpb_compact, dim3((tiles + 3) / 4), dim3(256), 0, c->stream, c->dwin());
    } else {
        hipLaunchKernelGGL(tw_lp_compact, dim3(compact_blocks(c->d.R)), dim3(256), 0, c->stream, c->dwin(), 0u, 0u);
    }
    HIPCHK(hipGetLastError());
    if (fuse) {
        hipLaunchKernelGGL(tw_lp_dmark, dim3(64), dim3(256), 0, c->stream, c->dwin());
        HIPCHK(hipGetLastError());
    } else if (bat) {
        hipLaunchKernelGGL(tw_lp_batch, dim3(TW_DUE_GRID), dim3(TW_BAT_T), 0, c->stream, c->dwin());
        HIPCHK(hipGetLastError());
    }
    return TW_OK;
}

int sh_lp_loop_begin(tw_shard* c) {
    if (!c) return TW_ERR_INVALID;
    if (!c->loaded || !c->lp) return TW_ERR_STATE;
    if (const char* b = getenv("TW_LP_TICK_BUDGET")) {
        const long v = strtol(b, nullptr, 10);
        c->lp_budget = v >= 1 && v <= (1 << 20) ? (uint32_t)v : (1u << 14);
    }
    if (const char* b = getenv("TW_LP_GRID")) {  // (tests: the grid-stride walk on small contexts)
        const long v = strtol(b, nullptr, 10);
        c->lp_grid = v >= 1 && v <= (1 << 20) ? (uint32_t)v : TW_LP_GRID;
    }
    HIPCHK(hipSetDevice(c->device));
    if (!c->ex_red) c->ex_red = c->red_own;  // world 1 without an explicit setup
    c->d.act_cur = 0;
    c->d.wid = 0;
    hipLaunchKernelGGL(tw_lp_begin, dim3(1), dim3(1), 0, c->stream, c->dwin(), c->d.lookahead);
    HIPCHK(hipGetLastError());
    // the record blocks' counts (tw_lp_ctl clears them every tick; a loop that
    // stopped inside a tick -- a failure on some rank -- may have left some)
    for (uint32_t g = 0; c->ex_send && g < c->ex_world; ++g)
        HIPCHK(hipMemsetAsync(c->ex_send + (size_t)g * (c->ex_cap + 1) * 2, 0, sizeof(uint4), c->stream));
    if (c->d.rw) {  // every replica's first window starts at 0; minima empty
        const size_t nrep = (size_t)1 << c->d.rep_lg;
        HIPCHK(hipMemsetAsync(c->d.rw + RW_T * nrep, 0, 8 * nrep, c->stream));
        HIPCHK(hipMemsetAsync(c->d.rw + RW_TICK * nrep, 0xFF, 8 * nrep * (RW_COUNT - RW_TICK), c->stream));
    }
    HIPCHK(hipMemsetAsync(c->d.lp_err, 0, 4, c->stream));
    if (c->d.dmk_n) HIPCHK(hipMemsetAsync(c->d.dmk_n, 0, 8, c->stream));
    int rc = lp_window_start(c);
    if (rc) return rc;
    c->loop_ready = true;
    return TW_OK;
}

static uint32_t lp_grid(uint32_t n) {
    const uint32_t b = (n + 255) / 256;
    return b < 1 ? 1 : b > 2048 ? 2048 : b;
}

int sh_lp_tick(tw_shard* c) {
    if (!c) return TW_ERR_INVALID;
    if (!c->loaded || !c->lp || !c->loop_ready) return TW_ERR_STATE;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    const Dev d = c->dwin();
    // the window comes from the device (tw_run_kernel reads c.win); launch
    // arguments are captured at enqueue, so d.win is set only around it
    c->d.win = c->win_buf;
    launch_run<true, TW_WG_LP, TW_NEAR_LP>(c, st, 0, UINT64_MAX, c->lp_budget);
    c->d.win = nullptr;
    HIPCHK(hipGetLastError());
    if (c->ex_world > 1 && d.carry) {  // the previous tick's carry claims block slots first
        hipLaunchKernelGGL(tw_lp_pack_carry, dim3(lp_grid(d.carry_cap)), dim3(256), 0, st, d, c->ex_send,
                           (const uint32_t*)c->ex_starts, c->ex_world, c->ex_cap, c->ex_cap_eff);
        HIPCHK(hipGetLastError());
    }
    hipLaunchKernelGGL(tw_lp_pack, dim3(lp_grid(d.out_cap)), dim3(256), 0, st, d, c->ex_send,
                       (const uint32_t*)c->ex_starts, c->ex_world, c->ex_cap, c->ex_cap_eff);
    HIPCHK(hipGetLastError());
    return TW_OK;
}

int sh_lp_tick_import(tw_shard* c) {
    if (!c) return TW_ERR_INVALID;
    if (!c->loaded || !c->lp || !c->loop_ready) return TW_ERR_STATE;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    // (no exchange buffers -- one rank of a caller-driven loop: tw_lp_ctl
    // fills the words itself)
    if (c->ex_send) {
        hipLaunchKernelGGL(tw_lp_import, dim3(lp_grid(c->ex_world * c->ex_cap_eff)), dim3(256), 0, st, c->dwin(),
                           (const uint4*)c->ex_recv, c->ex_world, c->ex_cap, c->ex_cap_eff);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(tw_lp_fill, dim3(1), dim3(1), 0, st, c->dwin(), c->ex_red, (const uint4*)c->ex_send,
                           c->ex_world, c->ex_cap);
        HIPCHK(hipGetLastError());
    }
    return TW_OK;
}

int sh_lp_tick_end(tw_shard* c) {
    if (!c) return TW_ERR_INVALID;
    if (!c->loaded || !c->lp || !c->loop_ready) return TW_ERR_STATE;
    HIPCHK(hipSetDevice(c->device));
    hipLaunchKernelGGL(tw_lp_ctl, dim3(1), dim3(1), 0, c->stream, c->dwin(), c->ex_red, c->ex_send, c->ex_world,
                       c->ex_cap, c->ex_send ? 1u : 0u);
    HIPCHK(hipGetLastError());
    if (c->d.rw) {
        const uint32_t nrep = 1u << c->d.rep_lg;
        hipLaunchKernelGGL(tw_lpb_rctl, dim3((nrep + 255) / 256), dim3(256), 0, c->stream, c->dwin());
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(tw_lpb_fin, dim3(1), dim3(1), 0, c->stream, c->dwin());
        HIPCHK(hipGetLastError());
    }
    return lp_window_start(c);
}

// the window words + lp_err into the pinned host copy (stream-ordered)
static int lp_progress_copy(tw_shard* c) {
    int64_t* w = c->h_win;  // pinned: plain DMA copies, no staging blit
    HIPCHK(hipMemcpyAsync(w, c->win_buf, 8 * WN_COUNT, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(w + WN_COUNT, c->d.lp_err, 4, hipMemcpyDeviceToHost, c->stream));
    return TW_OK;
}
static int lp_progress_read(tw_shard* c, tw_lp_state* out) {
    HIPCHK(hipStreamSynchronize(c->stream));
    const int64_t* w = c->h_win;
    const uint32_t err = (uint32_t)w[WN_COUNT];
    out->windows = (uint64_t)w[WN_WINDOWS];
    out->ticks = (uint64_t)w[WN_TICKS];
    out->t = w[WN_T];
    out->done = (w[WN_FLAGS] & WN_DONE) ? 1u : 0u;
    out->err = err;
    return TW_OK;
}
static int lp_host_alloc(tw_shard* c) {
    if (!c->h_win) HIPCHK(hipHostMalloc((void**)&c->h_win, 8 * (WN_COUNT + 1)));
    return TW_OK;
}

int sh_lp_progress(tw_shard* c, tw_lp_state* out) {
    if (!c || !out) return TW_ERR_INVALID;
    if (!c->loaded || !c->lp || !c->loop_ready) return TW_ERR_STATE;
    HIPCHK(hipSetDevice(c->device));
    int rc = lp_host_alloc(c);
    if (rc) return rc;
    c->h_win[WN_COUNT] = 0;  // lp_err fills its low 4 bytes
    rc = lp_progress_copy(c);
    return rc ? rc : lp_progress_read(c, out);
}

#define TW_GRAPH_TICKS 16
// the launch arguments a captured tick graph depends on
static std::vector<unsigned char> tick_key(const tw_shard* c) {
    struct K {
        Dev d;
        hipStream_t st;
        int64_t *win, *h_win, *red;
        uint4 *send, *recv;
        uint32_t *starts, budget, grid, world, cap, cap_eff;
        size_t lds;
        bool heavy;
    } k;
    std::memset(&k, 0, sizeof(k));
    std::memcpy(&k.d, &c->d, sizeof(Dev));
    k.st = c->stream;
    k.win = c->win_buf;
    k.h_win = c->h_win;
    k.red = c->ex_red;
    k.send = c->ex_send;
    k.recv = c->ex_recv;
    k.starts = c->ex_starts;
    k.budget = c->lp_budget;
    k.grid = c->lp_grid;
    k.world = c->ex_world;
    k.cap = c->ex_cap;
    k.cap_eff = c->ex_cap_eff;
    k.lds = c->lds_bytes;
    k.heavy = c->heavy_ok;
    std::vector<unsigned char> v(sizeof(K));
    std::memcpy(v.data(), &k, sizeof(K));
    return v;
}
// TW_GRAPH_TICKS ticks and the progress copy, captured once per set of launch
// arguments (every kernel of a tick reads its window from the device, so the
// same graph serves every batch; ticks after the loop is done return at once)
static int tick_graph_ready(tw_shard* c) {
    std::vector<unsigned char> key = tick_key(c);
    if (c->tick_graph && key == c->tick_gkey) return TW_OK;
    if (c->tick_graph) (void)hipGraphExecDestroy(c->tick_graph);
    c->tick_graph = nullptr;
    c->tick_gkey.clear();
    HIPCHK(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    int rc = TW_OK;
    for (int i = 0; i < TW_GRAPH_TICKS && !rc; ++i) {
        rc = sh_lp_tick(c);
        if (!rc) rc = sh_lp_tick_import(c);
        if (!rc) rc = sh_lp_tick_end(c);
    }
    if (!rc) rc = lp_progress_copy(c);
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(c->stream, &g);
    if (rc || e != hipSuccess) {
        if (g) (void)hipGraphDestroy(g);
        (void)hipGetLastError();
        return rc ? rc : TW_ERR_HIP;
    }
    const hipError_t ei = hipGraphInstantiate(&c->tick_graph, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (ei != hipSuccess) {
        c->tick_graph = nullptr;
        return TW_ERR_HIP;
    }
    c->tick_gkey = std::move(key);
    return TW_OK;
}

int sh_lp_run_windows(tw_shard* c, uint64_t max_ticks, tw_lp_state* out) {
    if (!c || !out) return TW_ERR_INVALID;
    if (!c->loaded || !c->lp || !c->loop_ready) return TW_ERR_STATE;
    if (c->ex_world != 1) return TW_ERR_STATE;
    HIPCHK(hipSetDevice(c->device));
    int rc = lp_host_alloc(c);
    if (rc) return rc;
    const char* ng = getenv("TW_NO_GRAPH");  // (A/B: launch every kernel from the host)
    const bool graph = !(ng && *ng && *ng != '0');
    for (uint64_t done_ticks = 0; done_ticks < max_ticks;) {
        const uint64_t batch =
            max_ticks - done_ticks < TW_GRAPH_TICKS ? max_ticks - done_ticks : (uint64_t)TW_GRAPH_TICKS;
        c->h_win[WN_COUNT] = 0;  // lp_err fills its low 4 bytes
        if (graph && batch == TW_GRAPH_TICKS) {
            rc = tick_graph_ready(c);
            if (rc) return rc;
            HIPCHK(hipGraphLaunch(c->tick_graph, c->stream));
        } else {
            for (uint64_t i = 0; i < batch; ++i) {
                rc = sh_lp_tick(c);
                if (!rc) rc = sh_lp_tick_import(c);
                if (!rc) rc = sh_lp_tick_end(c);
                if (rc) return rc;
            }
            rc = lp_progress_copy(c);
            if (rc) return rc;
        }
        done_ticks += batch;
        rc = lp_progress_read(c, out);
        if (rc) return rc;
        if (out->err) return TW_ERR_REPLICA;
        if (out->done) return TW_OK;
    }
    return TW_ERR_INCOMPLETE;
}

// Batched LP: tw_run = the whole device window loop (one host sync per 16 ticks)
static int lpb_run(tw_shard* c, tw_stats* out) {
    auto w0 = std::chrono::steady_clock::now();
    // the run's counts are the results minus those before it: zero right
    // after tw_reset (no reduction pass needed)
    std::vector<tw_replica_result> before;
    if (out) {
        before.resize(c->n_rep);
        if (c->lpb_fresh) {
            std::memset(before.data(), 0, sizeof(tw_replica_result) * before.size());
        } else {
            int rc = sh_read_results(c, before.data(), before.size());
            if (rc) return rc;
        }
    }
    c->lpb_fresh = false;
    while (c->ev_pool.size() < 2) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        c->ev_pool.push_back(e);
    }
    int rc = sh_lp_loop_begin(c);
    if (rc) return rc;
    HIPCHK(hipEventRecord(c->ev_pool[0], c->stream));
    tw_lp_state ls{};
    rc = sh_lp_run_windows(c, 1ull << 40, &ls);
    HIPCHK(hipEventRecord(c->ev_pool[1], c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, c->ev_pool[0], c->ev_pool[1]));
    c->launch_ms.assign(1, ms);
    c->lpb_windows = ls.windows;
    c->lpb_ticks = ls.ticks;
    if (rc) return rc;
    if (out) {
        std::memset(out, 0, sizeof(*out));
        std::vector<tw_replica_result> rr(c->n_rep);
        rc = sh_read_results(c, rr.data(), rr.size());
        if (rc) return rc;
        for (uint32_t i = 0; i < c->n_rep; ++i) {
            out->events += rr[i].events - before[i].events;
            out->delivered += rr[i].delivered - before[i].delivered;
            out->dropped += rr[i].dropped - before[i].dropped;
            out->undeliverable += rr[i].undeliverable - before[i].undeliverable;
            if (rr[i].final_t > out->max_final_t) out->max_final_t = rr[i].final_t;
            if (rr[i].status == TW_REP_DONE) ++out->replicas_done;
            if (rr[i].status >= TW_REP_ERR_SLOTS) ++out->replicas_error;
        }
        out->sends = out->delivered + out->dropped + out->undeliverable;
        out->launches = 1;  // the window loop, timed as one (tw_last_launch_ms)
        out->kernel_ms = ms;
        out->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
    }
    return TW_OK;
}

int sh_lpb_windows(tw_shard* c, uint64_t* windows, uint64_t* ticks) {
    if (!c) return TW_ERR_INVALID;
    if (!c->loaded || !c->lpb) return TW_ERR_STATE;
    if (windows) *windows = c->lpb_windows;
    if (ticks) *ticks = c->lpb_ticks;
    return TW_OK;
}

int sh_lpb_batch(tw_shard* c, uint64_t* batched, uint64_t* due) {
    if (!c) return TW_ERR_INVALID;
    if (!c->loaded || !c->lpb) return TW_ERR_STATE;
    unsigned long long h[2] = {0, 0};
    if (c->d.bat_ctr) {
        HIPCHK(hipSetDevice(c->device));
        HIPCHK(hipMemcpyAsync(h, c->d.bat_ctr, 16, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    if (batched) *batched = h[0];
    if (due) *due = h[1];
    return TW_OK;
}

// Diagnostic build only (-DTW_STATS): copy the P_COUNT counters out,
// optionally zeroing them; the product build has none (TW_ERR_STATE).
int sh_prof_read(tw_shard* c, unsigned long long* out, size_t cap, int reset) {
#ifdef TW_STATS
    if (!c || !out || !c->loaded || !c->d.prof) return TW_ERR_STATE;
    const size_t all = (size_t)2 * P_COUNT + TW_BPROF;  // all lanes, heavy LP lanes, tw_lp_batch's phases
    size_t n = cap < all ? cap : all;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpy(out, c->d.prof, 8 * n, hipMemcpyDeviceToHost));
    if (reset) HIPCHK(hipMemset(c->d.prof, 0, 8 * all));
    return (int)n;
#else
    (void)c; (void)out; (void)cap; (void)reset;
    return TW_ERR_STATE;
#endif
}

uint32_t sh_replicas(tw_shard* c) { return c->lpb ? c->n_rep : c->d.R; }
uint32_t sh_nodes(tw_shard* c) { return c->lpb ? c->d.Ntot : c->d.N; }
bool sh_is_lp(tw_shard* c) { return c->lp; }
int sh_device(tw_shard* c) { return c->device; }

int sh_set_trace(tw_shard* c, uint32_t cap) {
    if (!c) return TW_ERR_INVALID;
    if (!c->loaded) return TW_ERR_STATE;
    if (c->lp) return TW_ERR_INVALID;  // LP lanes are nodes: no replica execution order to record
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (c->d.trace) {
        HIPCHK(hipFree(c->d.trace));
        c->d.trace = nullptr;
    }
    c->d.trace_cap = 0;
    if (cap) {
        HIPCHK(hipMalloc(&c->d.trace, (size_t)cap * c->d.R * 32));
        c->d.trace_cap = cap;
    }
    return TW_OK;
}

int sh_read_trace(tw_shard* c, uint32_t replica, tw_trace_rec* out, size_t cap, uint64_t* n_emitted) {
    if (!c || (cap && !out)) return TW_ERR_INVALID;
    if (!c->loaded) return TW_ERR_STATE;
    const Dev& d = c->d;
    if (replica >= d.R) return TW_ERR_INVALID;
    HIPCHK(hipSetDevice(c->device));
    uint64_t n = 0;
    HIPCHK(hipMemcpyAsync(&n, d.scal + (size_t)SC_TRACE_N * d.R + replica, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (n_emitted) *n_emitted = n;
    size_t k = n < d.trace_cap ? (size_t)n : (size_t)d.trace_cap;
    if (k > cap) k = cap;
    if (k) {
        // records of one replica are strided by R: one 2D copy
        std::vector<uint4> buf(2 * k);
        HIPCHK(hipMemcpy2DAsync(buf.data(), 32, d.trace + (size_t)replica * 2, (size_t)d.R * 32, 32, k,
                                hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        for (size_t i = 0; i < k; ++i) {
            const uint4 a = buf[2 * i], b = buf[2 * i + 1];
            out[i].t = (int64_t)(((uint64_t)a.y << 32) | a.x);
            out[i].val = (int64_t)(((uint64_t)b.y << 32) | b.x);
            out[i].node = a.z;
            out[i].tag = a.w;
        }
    }
    return TW_OK;
}

int sh_last_launch_ms(tw_shard* c, double* out, size_t cap) {
    if (!c || !out) return TW_ERR_INVALID;
    size_t n = c->launch_ms.size() < cap ? c->launch_ms.size() : cap;
    for (size_t i = 0; i < n; ++i) out[i] = c->launch_ms[i];
    return (int)n;
}

}  // namespace tw
