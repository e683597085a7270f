// abi.hip — the public C ABI of libtimewarp.so (include/timewarp.h) over one
// or more device shards (engine.hip via shard.hpp).
//
// Replaces the runner of time-warp's pure-emulation path,
//   runTimedT :: (MonadIO m, MonadCatch m) => TimedT m a -> m a
//   (src/Control/TimeWarp/Timed/TimedT.hs:293-304),
// for a batch of replicas (or one node-partitioned scenario) spread over the
// GPUs of a node, with the library owning the collectives:
//   * tw_create(devices, ndev): one process drives ndev GPUs; replicas are
//     split into contiguous blocks [g*R/G, (g+1)*R/G), the
//     statistics are all-reduced over RCCL communicators the library creates
//     (ncclCommInitAll); a node-partitioned scenario's window loop moves its
//     record blocks by RCCL send/recv and reduces its window words by RCCL
//     all-reduce(min), all enqueued on the shards' streams.  A device listed
//     twice (tests on one GPU) or TW_TRANSPORT=copy uses device-to-device
//     copies ordered by HIP events instead of RCCL;
//   * tw_comm_id + tw_create_rank: one process per GPU (torchrun) with a
//     library-owned RCCL communicator over all ranks (ncclCommInitRank): the
//     same collectives, across processes.
// No CPU fallback: without a gfx950 device tw_create fails.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "../../include/timewarp.h"
#include "shard.hpp"
#include "tw_dev.hpp"

using namespace tw;

namespace {

enum Transport { TP_NONE, TP_RCCL, TP_COPY };

#define RD_N 4  // reduction words (tw_dev.hpp RD_COUNT)
static_assert(RD_N == RD_COUNT, "reduction words");

// COPY transport: red[i] = min over the ranks' words (staged in `all`)
__global__ void tw_red_min(int64_t* red, const int64_t* all, uint32_t world) {
    const uint32_t i = threadIdx.x;
    if (i >= RD_N) return;
    int64_t m = all[i];
    for (uint32_t g = 1; g < world; ++g) m = all[(size_t)g * RD_N + i] < m ? all[(size_t)g * RD_N + i] : m;
    red[i] = m;
}

}  // namespace

struct tw_ctx {
    std::vector<tw_shard*> sh;
    std::vector<int> dev;
    int world = 1;       // ranks of the job: this process's shards (tw_create) or the processes (tw_create_rank)
    int rank0 = 0;       // global rank of sh[0]
    Transport tp = TP_NONE;
    std::vector<ncclComm_t> comm;  // one per shard (TP_RCCL)
    std::vector<uint32_t> rep0;    // first replica of each shard, within this context
    // node-partitioned mode over several shards / ranks (tw_lp_run)
    uint32_t lp_begin = 0, lp_count = 0;
    bool lp_ready = false;                  // exchange buffers made for this load
    std::vector<uint32_t> starts;           // world + 1 node boundaries
    std::vector<int64_t*> red_all;          // COPY: per shard [world][RD_N]
    std::vector<hipEvent_t> ev_a, ev_b;     // COPY: per shard
    std::vector<void*> scratch;             // per shard: RCCL statistics buffer
    uint32_t xcap = 1u << 14;               // exchange block stride (records per rank pair)
    // an RCCL call of this context failed: the communicators may hold a
    // collective the peers are still in, so every later communicating call
    // returns TW_ERR_COMM without entering another one (timewarp.h, tw_lp_run)
    bool comm_broken = false;
    // testing hook (nccl_test_fail): TW_TEST_FAIL_NCCL as it was when the
    // context was made (0: off), and the checked RCCL calls made since
    long test_fail_at = 0;
    std::atomic<long> test_calls{0};
};

namespace {

int comm_fail(ncclResult_t r, const char* what) {
    fprintf(stderr, "timewarp: %s failed: %s\n", what, ncclGetErrorString(r));
    return TW_ERR_COMM;
}
// testing hook: a context made with TW_TEST_FAIL_NCCL=k in the environment
// fails its k-th checked RCCL call (counting from 1) without making it
// (one-rank jobs in the tests).  The variable is read once, when the context
// is made (test_hook_init), not on every call.
void test_hook_init(tw_ctx* c) {
    const char* e = getenv("TW_TEST_FAIL_NCCL");
    c->test_fail_at = e ? atol(e) : 0;
}
bool nccl_test_fail(tw_ctx* c) { return c->test_fail_at > 0 && ++c->test_calls == c->test_fail_at; }
// (in a function of the context c: a failure marks it unusable)
#define NCCLCHK(x)                                   \
    do {                                             \
        ncclResult_t _r = nccl_test_fail(c) ? ncclInternalError : (x); \
        if (_r != ncclSuccess) {                     \
            c->comm_broken = true;                   \
            return comm_fail(_r, #x);                \
        }                                            \
    } while (0)
// ... between ncclGroupStart and ncclGroupEnd: a failure closes the group
// first, so the thread is not left inside it (a later group of this thread --
// a fresh context's -- would be folded into the open one); the broken
// communicators are then aborted, not destroyed (destroy_parts)
#define NCCLCHK_G(x)                                 \
    do {                                             \
        ncclResult_t _r = nccl_test_fail(c) ? ncclInternalError : (x); \
        if (_r != ncclSuccess) {                     \
            (void)ncclGroupEnd();                    \
            c->comm_broken = true;                   \
            return comm_fail(_r, #x);                \
        }                                            \
    } while (0)
// ... the group's end: an injected failure still closes the group
#define NCCLCHK_GEND()                               \
    do {                                             \
        const bool _inj = nccl_test_fail(c);         \
        ncclResult_t _r = ncclGroupEnd();            \
        if (_inj) _r = ncclInternalError;            \
        if (_r != ncclSuccess) {                     \
            c->comm_broken = true;                   \
            return comm_fail(_r, "ncclGroupEnd()");  \
        }                                            \
    } while (0)
#define NCCLCHK_NC(x)                                \
    do {                                             \
        ncclResult_t _r = (x);                       \
        if (_r != ncclSuccess) return comm_fail(_r, #x); \
    } while (0)
#define HIPCHK_A(x)                                  \
    do {                                             \
        hipError_t _e = (x);                         \
        if (_e != hipSuccess) {                      \
            fprintf(stderr, "timewarp: %s failed: %s\n", #x, hipGetErrorString(_e)); \
            return _e == hipErrorOutOfMemory ? TW_ERR_OOM : TW_ERR_HIP; \
        }                                            \
    } while (0)

// run f(shard index) for every shard, concurrently when there are several
// (each shard is its own device and stream; the HIP runtime is thread-safe);
// returns the first error
template <class F>
int each_shard(tw_ctx* c, F f) {
    const size_t n = c->sh.size();
    if (n == 1) return f(0);
    std::vector<int> rc(n, TW_OK);
    std::vector<std::thread> th;
    th.reserve(n);
    for (size_t i = 0; i < n; ++i) th.emplace_back([&, i] { rc[i] = f(i); });
    for (auto& t : th) t.join();
    for (int r : rc)
        if (r != TW_OK) return r;
    return TW_OK;
}

int scratch_of(tw_ctx* c, size_t i, void** p) {
    if (c->scratch.size() != c->sh.size()) c->scratch.assign(c->sh.size(), nullptr);
    if (!c->scratch[i]) {
        HIPCHK_A(hipSetDevice(c->dev[i]));
        HIPCHK_A(hipMalloc(&c->scratch[i], 64 * 8));
    }
    *p = c->scratch[i];
    return TW_OK;
}

// All-reduce over the job (every shard of every rank): `sums` with SUM,
// `maxs` with MAX (int64), in place; one call per shard, enqueued as one
// RCCL group on the shards' streams.  Without RCCL the shards' values are
// combined on the host.
int job_reduce(tw_ctx* c, std::vector<std::vector<uint64_t>>& sums, std::vector<std::vector<int64_t>>& maxs) {
    const size_t n = c->sh.size();
    const size_t ns = sums[0].size(), nm = maxs[0].size();
    if (c->tp != TP_RCCL) {
        for (size_t i = 1; i < n; ++i) {
            for (size_t k = 0; k < ns; ++k) sums[0][k] += sums[i][k];
            for (size_t k = 0; k < nm; ++k) maxs[0][k] = std::max(maxs[0][k], maxs[i][k]);
        }
        for (size_t i = 1; i < n; ++i) { sums[i] = sums[0]; maxs[i] = maxs[0]; }
        return TW_OK;
    }
    std::vector<void*> buf(n);
    for (size_t i = 0; i < n; ++i) {
        int rc = scratch_of(c, i, &buf[i]);
        if (rc) return rc;
        HIPCHK_A(hipSetDevice(c->dev[i]));
        HIPCHK_A(hipMemcpy(buf[i], sums[i].data(), 8 * ns, hipMemcpyHostToDevice));
        HIPCHK_A(hipMemcpy((char*)buf[i] + 8 * ns, maxs[i].data(), 8 * nm, hipMemcpyHostToDevice));
    }
    NCCLCHK(ncclGroupStart());
    for (size_t i = 0; i < n; ++i) {
        NCCLCHK_G(ncclAllReduce(buf[i], buf[i], ns, ncclUint64, ncclSum, c->comm[i], nullptr));
        NCCLCHK_G(ncclAllReduce((char*)buf[i] + 8 * ns, (char*)buf[i] + 8 * ns, nm, ncclInt64, ncclMax, c->comm[i],
                              nullptr));
    }
    NCCLCHK_GEND();
    for (size_t i = 0; i < n; ++i) {
        HIPCHK_A(hipSetDevice(c->dev[i]));
        HIPCHK_A(hipStreamSynchronize(nullptr));
        HIPCHK_A(hipMemcpy(sums[i].data(), buf[i], 8 * ns, hipMemcpyDeviceToHost));
        HIPCHK_A(hipMemcpy(maxs[i].data(), (char*)buf[i] + 8 * ns, 8 * nm, hipMemcpyDeviceToHost));
    }
    return TW_OK;
}

// Status codes ranked by severity for the job-wide reduction (MAX): a hard
// runtime, communicator or state failure on one shard outranks a replica
// error or an incomplete run on another, whatever their numeric values
int64_t sev_of(int rc) {
    switch (rc) {
    case TW_OK: return 0;
    case TW_ERR_REPLICA: return 1;
    case TW_ERR_INCOMPLETE: return 2;
    case TW_ERR_INVALID: return 3;
    case TW_ERR_STATE: return 4;
    case TW_ERR_COMM: return 5;
    case TW_ERR_OOM: return 6;
    case TW_ERR_HIP: return 7;
    default: return 8;  // TW_ERR_NO_DEVICE and anything unknown
    }
}
int rc_of_sev(int64_t s) {
    static const int rcs[] = {TW_OK, TW_ERR_REPLICA, TW_ERR_INCOMPLETE, TW_ERR_INVALID, TW_ERR_STATE,
                              TW_ERR_COMM, TW_ERR_OOM, TW_ERR_HIP, TW_ERR_NO_DEVICE};
    return s >= 0 && s <= 8 ? rcs[s] : TW_ERR_HIP;
}

// Every shard of every rank learns the worst of the shards' local codes (one
// small all-reduce): a rank that failed locally joins the collective instead
// of leaving the others waiting in the next one
int job_agree(tw_ctx* c, const std::vector<int>& local, int* worst) {
    const size_t n = c->sh.size();
    std::vector<std::vector<uint64_t>> sums(n, std::vector<uint64_t>{0});
    std::vector<std::vector<int64_t>> maxs(n);
    for (size_t i = 0; i < n; ++i) maxs[i] = {sev_of(local[i])};
    const int rc = job_reduce(c, sums, maxs);
    if (rc) return rc;
    *worst = rc_of_sev(maxs[0][0]);
    return TW_OK;
}

int64_t dbits(double v) {
    int64_t b;
    std::memcpy(&b, &v, 8);
    return b;
}
double bitsd(int64_t b) {
    double v;
    std::memcpy(&v, &b, 8);
    return v;
}

// tw_stats of every shard -> the job's (sums of counts, max of times); the
// status code joins the reduction (the worst), so every rank returns it
int reduce_stats(tw_ctx* c, std::vector<tw_stats>& st, std::vector<int>& rcs, tw_stats* out, int* rc_out) {
    const size_t n = c->sh.size();
    std::vector<std::vector<uint64_t>> sums(n);
    std::vector<std::vector<int64_t>> maxs(n);
    for (size_t i = 0; i < n; ++i) {
        const tw_stats& s = st[i];
        sums[i] = {s.events, s.sends, s.delivered, s.dropped, s.undeliverable, s.replicas_done, s.replicas_error,
                   s.launches};
        maxs[i] = {s.max_final_t, dbits(s.kernel_ms), dbits(s.wall_ms), sev_of(rcs[i])};
    }
    int rc = job_reduce(c, sums, maxs);
    if (rc) return rc;
    if (out) {
        std::memset(out, 0, sizeof(*out));
        out->events = sums[0][0]; out->sends = sums[0][1]; out->delivered = sums[0][2]; out->dropped = sums[0][3];
        out->undeliverable = sums[0][4]; out->replicas_done = (uint32_t)sums[0][5];
        out->replicas_error = (uint32_t)sums[0][6]; out->launches = (uint32_t)sums[0][7];
        out->max_final_t = maxs[0][0]; out->kernel_ms = bitsd(maxs[0][1]); out->wall_ms = bitsd(maxs[0][2]);
    }
    *rc_out = rc_of_sev(maxs[0][3]);
    return TW_OK;
}

// a shard's slice of a replica batch: replicas [b0, b0 + nb) of desc, with
// the replica-minor link table and the main registers cut to them
struct SubDesc {
    tw_scenario_desc d;
    std::vector<uint32_t> table;
};
void sub_desc(const tw_scenario_desc* s, uint32_t b0, uint32_t nb, SubDesc& o) {
    o.d = *s;
    o.d.n_replicas = nb;
    if (s->main_regs) o.d.main_regs = s->main_regs + (size_t)b0 * 4;
    if (s->link_table) {
        const size_t rows = (size_t)s->n_links * s->link_depth;
        o.table.resize(rows * nb);
        for (size_t i = 0; i < rows; ++i)
            std::memcpy(o.table.data() + i * nb, s->link_table + i * s->n_replicas + b0, 4ull * nb);
        o.d.link_table = o.table.data();
    }
}

void split(uint32_t total, uint32_t parts, uint32_t i, uint32_t& b0, uint32_t& nb) {
    const uint32_t base = total / parts, rem = total % parts;
    b0 = i * base + std::min(i, rem);
    nb = base + (i < rem ? 1u : 0u);
}

int destroy_parts(tw_ctx* c) {
    // (a failed call may have left a collective the peers never joined:
    // abort, which does not wait for it, instead of destroy)
    for (size_t i = 0; i < c->comm.size(); ++i)
        if (c->comm[i]) (void)(c->comm_broken ? ncclCommAbort(c->comm[i]) : ncclCommDestroy(c->comm[i]));
    c->comm.clear();
    for (size_t i = 0; i < c->sh.size(); ++i) {
        (void)hipSetDevice(c->dev[i]);
        if (i < c->scratch.size() && c->scratch[i]) (void)hipFree(c->scratch[i]);
        if (i < c->red_all.size() && c->red_all[i]) (void)hipFree(c->red_all[i]);
        if (i < c->ev_a.size() && c->ev_a[i]) (void)hipEventDestroy(c->ev_a[i]);
        if (i < c->ev_b.size() && c->ev_b[i]) (void)hipEventDestroy(c->ev_b[i]);
        sh_destroy(c->sh[i]);
    }
    c->sh.clear();
    return TW_OK;
}

bool single(tw_ctx* c) { return c->sh.size() == 1; }

}  // namespace

static_assert(TW_ABI_VERSION == 4u, "tw_version names ABI 4");
static_assert(RD_N == TW_LP_RED_WORDS, "the caller-owned reduction buffer (timewarp.h)");

extern "C" {

const char* tw_version(void) {
    return "timewarp-mi355x 0.6 (gfx950; lane-per-replica dense/narrow/sparse kernels, wavefront-per-replica kernel, "
           "node-partitioned LP kernel with device-driven windows, batched logical processes (tw_lpb_load); "
           "multi-GPU contexts with library-owned RCCL communicators; "
           "ABI 4)";
}

const char* tw_strerror(int code) {
    switch (code) {
    case TW_OK: return "ok";
    case TW_ERR_INVALID: return "invalid argument or scenario descriptor";
    case TW_ERR_NO_DEVICE: return "no HIP device";
    case TW_ERR_HIP: return "HIP runtime error";
    case TW_ERR_OOM: return "device out of memory";
    case TW_ERR_STATE: return "call out of order";
    case TW_ERR_REPLICA: return "replica error";
    case TW_ERR_INCOMPLETE: return "relaunch cap reached before every replica stopped";
    case TW_ERR_COMM: return "RCCL error";
    default: return "unknown error";
    }
}

int tw_create(const int* devices, int ndev, tw_ctx** out) {
    if (!out) return TW_ERR_INVALID;
    *out = nullptr;
    if (!devices || ndev < 1 || ndev > 64) return TW_ERR_INVALID;
    tw_ctx* c = new (std::nothrow) tw_ctx;
    if (!c) return TW_ERR_OOM;
    for (int i = 0; i < ndev; ++i) {
        tw_shard* s = nullptr;
        int rc = sh_create(devices[i], &s);
        if (rc) {
            destroy_parts(c);
            delete c;
            return rc;
        }
        c->sh.push_back(s);
        c->dev.push_back(devices[i]);
    }
    c->world = ndev;
    c->rank0 = 0;
    test_hook_init(c);
    if (ndev > 1) {
        std::vector<int> sorted(c->dev);
        std::sort(sorted.begin(), sorted.end());
        const bool dup = std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end();
        const char* t = getenv("TW_TRANSPORT");
        c->tp = (dup || (t && !strcmp(t, "copy"))) ? TP_COPY : TP_RCCL;
        if (c->tp == TP_RCCL) {
            c->comm.assign(ndev, nullptr);
            const ncclResult_t r = ncclCommInitAll(c->comm.data(), ndev, c->dev.data());
            if (r != ncclSuccess) {
                comm_fail(r, "ncclCommInitAll");
                c->comm.assign(ndev, nullptr);
                destroy_parts(c);
                delete c;
                return TW_ERR_COMM;
            }
        }
    }
    *out = c;
    return TW_OK;
}

int tw_comm_id(uint8_t* id) {
    if (!id) return TW_ERR_INVALID;
    ncclUniqueId u;
    NCCLCHK_NC(ncclGetUniqueId(&u));
    static_assert(sizeof(u) == TW_COMM_ID_BYTES, "RCCL unique id size");
    std::memcpy(id, &u, sizeof(u));
    return TW_OK;
}

int tw_create_rank(int device, int nranks, int rank, const uint8_t* id, tw_ctx** out) {
    if (!out) return TW_ERR_INVALID;
    *out = nullptr;
    if (!id || nranks < 1 || rank < 0 || rank >= nranks) return TW_ERR_INVALID;
    tw_ctx* c = new (std::nothrow) tw_ctx;
    if (!c) return TW_ERR_OOM;
    tw_shard* s = nullptr;
    int rc = sh_create(device, &s);
    if (rc) {
        delete c;
        return rc;
    }
    c->sh.push_back(s);
    c->dev.push_back(device);
    c->world = nranks;
    c->rank0 = rank;
    c->tp = TP_RCCL;
    test_hook_init(c);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    c->comm.assign(1, nullptr);
    (void)hipSetDevice(device);
    const ncclResult_t r = ncclCommInitRank(&c->comm[0], nranks, u, rank);
    if (r != ncclSuccess) {
        comm_fail(r, "ncclCommInitRank");
        c->comm.assign(1, nullptr);
        destroy_parts(c);
        delete c;
        return TW_ERR_COMM;
    }
    *out = c;
    return TW_OK;
}

int tw_ctx_info(tw_ctx* c, int* ndev, int* world, int* rank0, int* transport) {
    if (!c) return TW_ERR_INVALID;
    if (ndev) *ndev = (int)c->sh.size();
    if (world) *world = c->world;
    if (rank0) *rank0 = c->rank0;
    if (transport) *transport = (int)c->tp;
    return TW_OK;
}

void tw_destroy(tw_ctx* c) {
    if (!c) return;
    destroy_parts(c);
    delete c;
}

// ------------------------------------------------------------ replica mode
static int load_split(tw_ctx* c, const tw_scenario_desc* s, bool pow2,
                      int (*ld)(tw_shard*, const tw_scenario_desc*, const void*), const void* arg) {
    const uint32_t n = (uint32_t)c->sh.size();
    if (!s || s->n_replicas < n) return TW_ERR_INVALID;
    if (pow2) {  // batched LP: every shard's block a power of two
        if (s->n_replicas % n) return TW_ERR_INVALID;
        const uint32_t b = s->n_replicas / n;
        if (b & (b - 1)) return TW_ERR_INVALID;
    }
    c->rep0.assign(n, 0);
    std::vector<SubDesc> sd(n);
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t b0, nb;
        split(s->n_replicas, n, i, b0, nb);
        c->rep0[i] = b0;
        sub_desc(s, b0, nb, sd[i]);
    }
    return each_shard(c, [&](size_t i) { return ld(c->sh[i], &sd[i].d, arg); });
}

int tw_load(tw_ctx* c, const tw_scenario_desc* s) {
    if (!c) return TW_ERR_INVALID;
    c->lp_ready = false;
    if (single(c)) {
        c->rep0.assign(1, 0);
        return sh_load(c->sh[0], s);
    }
    return load_split(c, s, false, [](tw_shard* h, const tw_scenario_desc* d, const void*) { return sh_load(h, d); },
                      nullptr);
}

int tw_reset(tw_ctx* c) {
    if (!c) return TW_ERR_INVALID;
    for (tw_shard* s : c->sh) {
        int rc = sh_reset(s);
        if (rc) return rc;
    }
    return TW_OK;
}

int tw_run(tw_ctx* c, int64_t t_end_us, uint64_t max_events, tw_stats* out) {
    if (!c) return TW_ERR_INVALID;
    if (single(c) && c->tp == TP_NONE) return sh_run(c->sh[0], t_end_us, max_events, out);
    if (c->comm_broken) return TW_ERR_COMM;
    const size_t n = c->sh.size();
    std::vector<tw_stats> st(n);
    std::vector<int> rcs(n, TW_OK);
    auto w0 = std::chrono::steady_clock::now();
    (void)each_shard(c, [&](size_t i) {
        rcs[i] = sh_run(c->sh[i], t_end_us, max_events, &st[i]);
        return TW_OK;
    });
    for (size_t i = 0; i < n; ++i)
        if (rcs[i] != TW_OK && rcs[i] != TW_ERR_INCOMPLETE && rcs[i] != TW_ERR_REPLICA) std::memset(&st[i], 0, sizeof(tw_stats));
    int rc = TW_OK;
    tw_stats agg{};
    int e = reduce_stats(c, st, rcs, &agg, &rc);
    if (e) return e;
    agg.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
    if (out) *out = agg;
    return rc;
}

int tw_tie_audit(tw_ctx* c, int64_t t_end_us, uint64_t max_events, uint32_t probes, tw_stats* out) {
    if (!c) return TW_ERR_INVALID;
    if (single(c) && c->tp == TP_NONE) return sh_tie_audit(c->sh[0], t_end_us, max_events, probes, out);
    if (c->comm_broken) return TW_ERR_COMM;
    const size_t n = c->sh.size();
    std::vector<tw_stats> st(n);
    std::vector<int> rcs(n, TW_OK);
    (void)each_shard(c, [&](size_t i) {
        rcs[i] = sh_tie_audit(c->sh[i], t_end_us, max_events, probes, &st[i]);
        return TW_OK;
    });
    int rc = TW_OK;
    int e = reduce_stats(c, st, rcs, out, &rc);
    return e ? e : rc;
}

static size_t local_replicas(tw_ctx* c) {
    size_t n = 0;
    for (tw_shard* s : c->sh) n += sh_replicas(s);
    return n;
}

int tw_read_results(tw_ctx* c, tw_replica_result* out, size_t n) {
    if (!c || !out) return TW_ERR_INVALID;
    if (n < local_replicas(c)) return TW_ERR_INVALID;
    size_t off = 0;
    for (tw_shard* s : c->sh) {
        const size_t k = sh_replicas(s);
        int rc = sh_read_results(s, out + off, k);
        if (rc) return rc;
        off += k;
    }
    return TW_OK;
}

int tw_read_hashes(tw_ctx* c, uint64_t* out, size_t n) {
    if (!c || !out) return TW_ERR_INVALID;
    size_t need = 0;
    for (tw_shard* s : c->sh) need += (size_t)sh_replicas(s) * sh_nodes(s);
    if (n < need) return TW_ERR_INVALID;
    size_t off = 0;
    for (tw_shard* s : c->sh) {
        const size_t k = (size_t)sh_replicas(s) * sh_nodes(s);
        int rc = sh_read_hashes(s, out + off, k);
        if (rc) return rc;
        off += k;
    }
    return TW_OK;
}

int tw_read_final(tw_ctx* c, int64_t* max_final_t, uint64_t* delivered, uint64_t* dropped, uint64_t* events) {
    if (!c) return TW_ERR_INVALID;
    std::vector<tw_replica_result> rr(local_replicas(c));
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

int tw_set_trace(tw_ctx* c, uint32_t cap) {
    if (!c) return TW_ERR_INVALID;
    for (tw_shard* s : c->sh) {
        int rc = sh_set_trace(s, cap);
        if (rc) return rc;
    }
    return TW_OK;
}

int tw_read_trace(tw_ctx* c, uint32_t replica, tw_trace_rec* out, size_t cap, uint64_t* n_emitted) {
    if (!c) return TW_ERR_INVALID;
    for (size_t i = c->sh.size(); i-- > 0;) {
        const uint32_t b0 = i < c->rep0.size() ? c->rep0[i] : 0u;
        if (replica >= b0) return sh_read_trace(c->sh[i], replica - b0, out, cap, n_emitted);
    }
    return TW_ERR_INVALID;
}

int tw_set_counter_base(tw_ctx* c, uint32_t seq0, uint32_t tid0) {
    if (!c) return TW_ERR_INVALID;
    for (tw_shard* s : c->sh) {
        int rc = sh_set_counter_base(s, seq0, tid0);
        if (rc) return rc;
    }
    return TW_OK;
}

int tw_set_tie_mode(tw_ctx* c, uint32_t mode) {
    if (!c) return TW_ERR_INVALID;
    for (tw_shard* s : c->sh) {
        int rc = sh_set_tie_mode(s, mode);
        if (rc) return rc;
    }
    return TW_OK;
}

int tw_geometry(tw_ctx* c) {
    if (!c) return TW_ERR_INVALID;
    return sh_geometry(c->sh[0]);
}

int tw_last_launch_ms(tw_ctx* c, double* out, size_t cap) {
    if (!c || !out) return TW_ERR_INVALID;
    size_t n = 0;
    for (tw_shard* s : c->sh) {
        int k = sh_last_launch_ms(s, out + n, cap - n);
        if (k < 0) return k;
        n += (size_t)k;
    }
    return (int)n;
}

// ------------------------------------------------- node-partitioned (LP) mode
int tw_lp_load(tw_ctx* c, const tw_scenario_desc* s, uint32_t lp_begin, uint32_t lp_count, int64_t lookahead_us,
               uint32_t inbox_cap, uint32_t outbox_cap) {
    if (!c || !s) return TW_ERR_INVALID;
    c->lp_ready = false;
    c->lp_begin = lp_begin;
    c->lp_count = lp_count;
    const uint32_t n = (uint32_t)c->sh.size();
    if (n == 1) return sh_lp_load(c->sh[0], s, lp_begin, lp_count, lookahead_us, inbox_cap, outbox_cap);
    if (lp_count < n) return TW_ERR_INVALID;
    return each_shard(c, [&](size_t i) {
        uint32_t b0, nb;
        split(lp_count, n, (uint32_t)i, b0, nb);
        return sh_lp_load(c->sh[i], s, lp_begin + b0, nb, lookahead_us, inbox_cap, outbox_cap);
    });
}

int tw_lpb_load(tw_ctx* c, const tw_scenario_desc* s, int64_t lookahead_us, const uint32_t* node_inbox_cap,
                uint32_t inbox_cap, uint32_t outbox_cap) {
    if (!c) return TW_ERR_INVALID;
    c->lp_ready = false;
    if (single(c)) {
        c->rep0.assign(1, 0);
        return sh_lpb_load(c->sh[0], s, lookahead_us, node_inbox_cap, inbox_cap, outbox_cap);
    }
    struct A { int64_t L; const uint32_t* caps; uint32_t ib, ob; } a{lookahead_us, node_inbox_cap, inbox_cap, outbox_cap};
    return load_split(c, s, true,
                      [](tw_shard* h, const tw_scenario_desc* d, const void* p) {
                          const A* q = (const A*)p;
                          return sh_lpb_load(h, d, q->L, q->caps, q->ib, q->ob);
                      },
                      &a);
}

int tw_lpb_windows(tw_ctx* c, uint64_t* windows, uint64_t* ticks) {
    if (!c) return TW_ERR_INVALID;
    uint64_t w = 0, t = 0;
    for (tw_shard* s : c->sh) {
        uint64_t a = 0, b = 0;
        int rc = sh_lpb_windows(s, &a, &b);
        if (rc) return rc;
        w = std::max(w, a);
        t = std::max(t, b);
    }
    if (windows) *windows = w;
    if (ticks) *ticks = t;
    return TW_OK;
}

int tw_lpb_batch(tw_ctx* c, uint64_t* batched, uint64_t* due_records) {
    if (!c) return TW_ERR_INVALID;
    uint64_t b = 0, d = 0;
    for (tw_shard* s : c->sh) {
        uint64_t x = 0, y = 0;
        int rc = sh_lpb_batch(s, &x, &y);
        if (rc) return rc;
        b += x;
        d += y;
    }
    if (batched) *batched = b;
    if (due_records) *due_records = d;
    return TW_OK;
}

// the host-driven window loop and the caller-driven device loop speak for one
// shard (the caller moves the records between contexts / ranks)
#define ONE_SHARD(c)                                  \
    do {                                              \
        if (!(c)) return TW_ERR_INVALID;              \
        if (!single(c)) return TW_ERR_STATE;          \
    } while (0)

int tw_lp_window(tw_ctx* c, int64_t t_end_excl, int64_t* next_t, uint64_t* n_foreign) {
    ONE_SHARD(c);
    return sh_lp_window(c->sh[0], t_end_excl, next_t, n_foreign);
}
int tw_lp_take_outbox(tw_ctx* c, tw_lp_record* out, size_t cap, size_t* n) {
    ONE_SHARD(c);
    return sh_lp_take_outbox(c->sh[0], out, cap, n);
}
int tw_lp_inject(tw_ctx* c, const tw_lp_record* recs, size_t n, int64_t* next_t) {
    ONE_SHARD(c);
    return sh_lp_inject(c->sh[0], recs, n, next_t);
}
int tw_set_stream(tw_ctx* c, void* hs) {
    ONE_SHARD(c);
    return sh_set_stream(c->sh[0], hs);
}
int tw_lp_exchange_setup(tw_ctx* c, uint32_t world, uint32_t rank, const uint32_t* starts, void* send, void* recv,
                         uint32_t cap, int64_t* red) {
    ONE_SHARD(c);
    c->lp_ready = false;
    return sh_lp_exchange_setup(c->sh[0], world, rank, starts, send, recv, cap, red);
}
int tw_lp_loop_begin(tw_ctx* c) {
    ONE_SHARD(c);
    return sh_lp_loop_begin(c->sh[0]);
}
int tw_lp_tick(tw_ctx* c) {
    ONE_SHARD(c);
    return sh_lp_tick(c->sh[0]);
}
int tw_lp_tick_import(tw_ctx* c) {
    ONE_SHARD(c);
    return sh_lp_tick_import(c->sh[0]);
}
int tw_lp_tick_end(tw_ctx* c) {
    ONE_SHARD(c);
    return sh_lp_tick_end(c->sh[0]);
}
int tw_lp_progress(tw_ctx* c, tw_lp_state* out) {
    ONE_SHARD(c);
    return sh_lp_progress(c->sh[0], out);
}
int tw_lp_run_windows(tw_ctx* c, uint64_t max_ticks, tw_lp_state* out) {
    ONE_SHARD(c);
    return sh_lp_run_windows(c->sh[0], max_ticks, out);
}

// Results of a node-partitioned run: the whole job's (every shard of every
// rank: counts summed, final time / status / main exception the largest,
// node hashes summed mod 2^64).
int tw_lp_results(tw_ctx* c, tw_replica_result* agg, uint64_t* node_hashes, size_t n_nodes) {
    if (!c || !agg) return TW_ERR_INVALID;
    if (single(c) && c->tp == TP_NONE) return sh_lp_results(c->sh[0], agg, node_hashes, n_nodes);
    if (c->comm_broken) return TW_ERR_COMM;
    const size_t n = c->sh.size();
    std::vector<std::vector<uint64_t>> sums(n);
    std::vector<std::vector<int64_t>> maxs(n);
    std::vector<std::vector<uint64_t>> hs(n);
    for (size_t i = 0; i < n; ++i) {
        tw_replica_result a{};
        hs[i].assign(n_nodes, 0);
        // a local failure joins the reduction (every rank returns it) instead
        // of leaving the other ranks in the all-reduce
        const int lrc = sh_lp_results(c->sh[i], &a, node_hashes ? hs[i].data() : nullptr, n_nodes);
        sums[i] = {a.events, a.delivered, a.dropped, a.undeliverable, a.threads};
        maxs[i] = {a.final_t, (int64_t)a.status, (int64_t)a.main_exc, sev_of(lrc)};
    }
    int rc = job_reduce(c, sums, maxs);
    if (rc) return rc;
    if (maxs[0][3]) return rc_of_sev(maxs[0][3]);
    std::memset(agg, 0, sizeof(*agg));
    agg->events = sums[0][0]; agg->delivered = sums[0][1]; agg->dropped = sums[0][2];
    agg->undeliverable = sums[0][3]; agg->threads = sums[0][4];
    agg->final_t = maxs[0][0]; agg->status = (uint32_t)maxs[0][1]; agg->main_exc = (uint32_t)maxs[0][2];
    if (node_hashes) {
        if (c->tp == TP_RCCL) {
            std::vector<void*> buf(n);
            for (size_t i = 0; i < n; ++i) {
                HIPCHK_A(hipSetDevice(c->dev[i]));
                HIPCHK_A(hipMalloc(&buf[i], 8 * n_nodes + 8));
                HIPCHK_A(hipMemcpy(buf[i], hs[i].data(), 8 * n_nodes, hipMemcpyHostToDevice));
            }
            NCCLCHK(ncclGroupStart());
            for (size_t i = 0; i < n; ++i)
                NCCLCHK_G(ncclAllReduce(buf[i], buf[i], n_nodes, ncclUint64, ncclSum, c->comm[i], nullptr));
            NCCLCHK_GEND();
            for (size_t i = 0; i < n; ++i) {
                HIPCHK_A(hipSetDevice(c->dev[i]));
                HIPCHK_A(hipStreamSynchronize(nullptr));
                if (i == 0) HIPCHK_A(hipMemcpy(node_hashes, buf[i], 8 * n_nodes, hipMemcpyDeviceToHost));
                HIPCHK_A(hipFree(buf[i]));
            }
        } else {
            for (size_t k = 0; k < n_nodes; ++k) {
                uint64_t h = 0;
                for (size_t i = 0; i < n; ++i) h += hs[i][k];
                node_hashes[k] = h;
            }
        }
    }
    return TW_OK;
}

// The whole device window loop of a node-partitioned scenario from t = 0 (after
// tw_reset), over every shard and rank, with the exchange the library owns:
// per tick every shard's event kernel + packing, then the record blocks
// between ranks (RCCL send/recv, or device copies), the import, the
// all-reduce(min) of the window words (RCCL, or a device min), the advance.
// Blocks travel at the size the ranks last agreed on (the largest per-rank
// demand of a tick, rounded up, re-chosen every 16 ticks from the reduced
// words, so every rank picks the same); records beyond it wait a tick in the
// carry buffer.  One host synchronisation per 16 ticks.
int tw_lp_run(tw_ctx* c, uint64_t max_ticks, tw_lp_state* out) {
    if (!c || !out) return TW_ERR_INVALID;
    if (c->comm_broken) return TW_ERR_COMM;
    const size_t n = c->sh.size();
    std::vector<int> lrc(n, TW_OK);  // each shard's first local failure
    // the worst local code of the job (RCCL: agreed over every rank first)
    auto agreed = [&](int* worst) -> int {
        if (c->tp != TP_RCCL) {
            int w = TW_OK;
            for (int r : lrc)
                if (sev_of(r) > sev_of(w)) w = r;
            *worst = w;
            return TW_OK;
        }
        return job_agree(c, lrc, worst);
    };
    for (tw_shard* s : c->sh)
        if (!sh_is_lp(s)) return TW_ERR_STATE;
    if (n == 1 && c->tp == TP_NONE) {
        // one context, no transport: the shard's own loop
        const uint32_t st2[2] = {c->lp_begin, c->lp_begin + c->lp_count};
        int rc = sh_lp_exchange_setup(c->sh[0], 1, 0, st2, nullptr, nullptr, 0, nullptr);
        if (!rc) rc = sh_lp_loop_begin(c->sh[0]);
        if (!rc) rc = sh_lp_run_windows(c->sh[0], max_ticks, out);
        return rc;
    }
    if (!c->lp_ready) {
        // node boundaries of every rank
        c->starts.assign((size_t)c->world + 1, 0);
        if (c->tp == TP_RCCL && n == 1 && c->world > 1) {
            // one shard per process: all-gather (begin, count) over the ranks
            void* buf = nullptr;
            HIPCHK_A(hipSetDevice(c->dev[0]));
            HIPCHK_A(hipMalloc(&buf, 8ull * (c->world + 1)));
            const uint32_t mine[2] = {c->lp_begin, c->lp_count};
            HIPCHK_A(hipMemcpy((char*)buf + 8ull * c->world, mine, 8, hipMemcpyHostToDevice));
            NCCLCHK(ncclAllGather((char*)buf + 8ull * c->world, buf, 2, ncclUint32, c->comm[0], nullptr));
            HIPCHK_A(hipStreamSynchronize(nullptr));
            std::vector<uint32_t> h(2ull * c->world);
            HIPCHK_A(hipMemcpy(h.data(), buf, 8ull * c->world, hipMemcpyDeviceToHost));
            HIPCHK_A(hipFree(buf));
            for (int g = 0; g < c->world; ++g) {
                c->starts[g] = h[2 * g];
                if (g > 0 && h[2 * g] != h[2 * (g - 1)] + h[2 * (g - 1) + 1]) return TW_ERR_INVALID;  // not contiguous
            }
            c->starts[c->world] = h[2 * (c->world - 1)] + h[2 * (c->world - 1) + 1];
        } else {
            for (int g = 0; g < c->world; ++g) {
                uint32_t b0, nb;
                split(c->lp_count, (uint32_t)c->world, (uint32_t)g, b0, nb);
                c->starts[g] = c->lp_begin + b0;
            }
            c->starts[c->world] = c->lp_begin + c->lp_count;
        }
        if (const char* x = getenv("TW_LP_XCAP")) {
            const long v = strtol(x, nullptr, 10);
            if (v >= 1 && v <= (1 << 22)) c->xcap = (uint32_t)v;
        }
        // (a shard's local failure from here on is carried to every rank by
        // job_agree before the next collective: no rank is left waiting in one)
        for (size_t i = 0; i < n; ++i)
            if (!lrc[i]) lrc[i] = sh_lp_exchange_own(c->sh[i], (uint32_t)c->world, (uint32_t)(c->rank0 + i),
                                                     c->starts.data(), c->xcap);
        if (c->tp == TP_COPY) {
            c->red_all.assign(n, nullptr);
            c->ev_a.assign(n, nullptr);
            c->ev_b.assign(n, nullptr);
            for (size_t i = 0; i < n; ++i) {
                HIPCHK_A(hipSetDevice(c->dev[i]));
                HIPCHK_A(hipMalloc((void**)&c->red_all[i], 8ull * RD_N * c->world));
                HIPCHK_A(hipEventCreateWithFlags(&c->ev_a[i], hipEventDisableTiming));
                HIPCHK_A(hipEventCreateWithFlags(&c->ev_b[i], hipEventDisableTiming));
            }
        }
        c->lp_ready = true;
    }
    std::vector<ShardXchg> x(n);
    uint32_t cap_eff = 0;
    for (size_t i = 0; i < n; ++i) {
        if (!lrc[i]) lrc[i] = sh_lp_loop_begin(c->sh[i]);
        if (!lrc[i]) sh_lp_exchange_info(c->sh[i], &x[i]);
        if (!lrc[i]) cap_eff = std::min<uint32_t>(x[i].stride, 4096u);
    }
    for (size_t i = 0; i < n; ++i)
        if (!lrc[i]) lrc[i] = sh_lp_set_block(c->sh[i], cap_eff);
    {
        int worst = TW_OK;
        const int rc = agreed(&worst);
        if (rc) return rc;
        if (worst) {
            if (c->lp_ready) c->lp_ready = false;  // (set up again by the next call)
            return worst;
        }
    }
    const size_t stride_b = 32ull * ((size_t)x[0].stride + 1);
    std::vector<tw_lp_state> st(n);
    // testing hook: TW_TEST_FAIL_TICK=shard:tick makes that local shard's
    // launches at that tick fail (TW_ERR_STATE), as a HIP or launch error
    // would -- the other shards and ranks must still leave together
    long fail_sh = -1, fail_tk = -1;
    if (const char* f = getenv("TW_TEST_FAIL_TICK")) {
        char* e = nullptr;
        fail_sh = strtol(f, &e, 10);
        fail_tk = (e && *e == ':') ? strtol(e + 1, nullptr, 10) : -1;
    }
    for (uint64_t done_ticks = 0; done_ticks < max_ticks;) {
        const uint64_t batch = std::min<uint64_t>(max_ticks - done_ticks, 16);
        const size_t bytes = 32ull * ((size_t)cap_eff + 1);
        for (uint64_t k = 0; k < batch; ++k) {
            // a shard that failed stops launching but keeps taking part in the
            // exchange and the reduction until the batch's agreement
            for (size_t i = 0; i < n; ++i) {
                if (!lrc[i]) lrc[i] = sh_lp_tick(c->sh[i]);
                if (!lrc[i] && (long)i == fail_sh && (long)(done_ticks + k) == fail_tk) lrc[i] = TW_ERR_STATE;
            }
            // record blocks: block g of rank r's send -> block r of rank g's recv
            if (c->tp == TP_RCCL) {
                NCCLCHK(ncclGroupStart());
                for (size_t i = 0; i < n; ++i)
                    for (int g = 0; g < c->world; ++g) {
                        NCCLCHK_G(ncclSend((char*)x[i].send + g * stride_b, bytes, ncclUint8, g, c->comm[i], x[i].stream));
                        NCCLCHK_G(ncclRecv((char*)x[i].recv + g * stride_b, bytes, ncclUint8, g, c->comm[i], x[i].stream));
                    }
                NCCLCHK_GEND();
            } else {
                for (size_t i = 0; i < n; ++i) {
                    HIPCHK_A(hipSetDevice(c->dev[i]));
                    HIPCHK_A(hipEventRecord(c->ev_a[i], x[i].stream));
                }
                for (size_t i = 0; i < n; ++i) {
                    HIPCHK_A(hipSetDevice(c->dev[i]));
                    for (size_t g = 0; g < n; ++g) {
                        if (g != i) HIPCHK_A(hipStreamWaitEvent(x[i].stream, c->ev_a[g], 0));
                        char* dst = (char*)x[i].recv + g * stride_b;
                        const char* src = (const char*)x[g].send + i * stride_b;
                        if (c->dev[g] == c->dev[i])
                            HIPCHK_A(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, x[i].stream));
                        else
                            HIPCHK_A(hipMemcpyPeerAsync(dst, c->dev[i], src, c->dev[g], bytes, x[i].stream));
                    }
                }
            }
            for (size_t i = 0; i < n; ++i)
                if (!lrc[i]) lrc[i] = sh_lp_tick_import(c->sh[i]);
            // window words: all-reduce(min)
            if (c->tp == TP_RCCL) {
                NCCLCHK(ncclGroupStart());
                for (size_t i = 0; i < n; ++i)
                    NCCLCHK_G(ncclAllReduce(x[i].red, x[i].red, RD_N, ncclInt64, ncclMin, c->comm[i], x[i].stream));
                NCCLCHK_GEND();
            } else {
                for (size_t i = 0; i < n; ++i) {
                    HIPCHK_A(hipSetDevice(c->dev[i]));
                    HIPCHK_A(hipEventRecord(c->ev_b[i], x[i].stream));
                }
                for (size_t i = 0; i < n; ++i) {
                    HIPCHK_A(hipSetDevice(c->dev[i]));
                    for (size_t g = 0; g < n; ++g) {
                        if (g != i) HIPCHK_A(hipStreamWaitEvent(x[i].stream, c->ev_b[g], 0));
                        if (c->dev[g] == c->dev[i])
                            HIPCHK_A(hipMemcpyAsync(c->red_all[i] + g * RD_N, x[g].red, 8 * RD_N,
                                                    hipMemcpyDeviceToDevice, x[i].stream));
                        else
                            HIPCHK_A(hipMemcpyPeerAsync(c->red_all[i] + g * RD_N, c->dev[i], x[g].red, c->dev[g],
                                                        8 * RD_N, x[i].stream));
                    }
                }
                // every shard's copies of the others' words must land before any
                // shard overwrites its own (its next tick's fill): a second event
                // round orders the min after all copies
                for (size_t i = 0; i < n; ++i) {
                    HIPCHK_A(hipSetDevice(c->dev[i]));
                    HIPCHK_A(hipEventRecord(c->ev_a[i], x[i].stream));
                }
                for (size_t i = 0; i < n; ++i) {
                    HIPCHK_A(hipSetDevice(c->dev[i]));
                    for (size_t g = 0; g < n; ++g)
                        if (g != i) HIPCHK_A(hipStreamWaitEvent(x[i].stream, c->ev_a[g], 0));
                    hipLaunchKernelGGL(tw_red_min, dim3(1), dim3(64), 0, x[i].stream, x[i].red,
                                       (const int64_t*)c->red_all[i], (uint32_t)n);
                    HIPCHK_A(hipGetLastError());
                }
            }
            for (size_t i = 0; i < n; ++i)
                if (!lrc[i]) lrc[i] = sh_lp_tick_end(c->sh[i]);
        }
        done_ticks += batch;
        bool err = false, done = true;
        for (size_t i = 0; i < n; ++i) {
            if (!lrc[i]) lrc[i] = sh_lp_progress(c->sh[i], &st[i]);
            err = err || st[i].err;
            done = done && st[i].done;
        }
        {
            int worst = TW_OK;
            const int rc = agreed(&worst);
            if (rc) return rc;
            if (worst) return worst;
        }
        *out = st[0];
        for (size_t i = 1; i < n; ++i) out->err |= st[i].err;
        if (err) return TW_ERR_REPLICA;
        if (done) return TW_OK;
        // the next batch's block size, from the largest demand any rank had in
        // one tick (reduced, so identical on every rank)
        const int64_t dem = sh_lp_xmax(c->sh[0]);
        uint32_t want = 64;
        while (want < (uint64_t)dem + (uint64_t)dem / 4 && want < x[0].stride) want <<= 1;
        want = std::min(want, x[0].stride);
        if (want > cap_eff || want * 4 <= cap_eff) cap_eff = want;
        for (size_t i = 0; i < n; ++i) {
            if (!lrc[i]) lrc[i] = sh_lp_set_block(c->sh[i], cap_eff);
            if (!lrc[i]) lrc[i] = sh_lp_clear_xmax(c->sh[i]);
        }
    }
    int worst = TW_OK;
    const int rc = agreed(&worst);
    if (rc) return rc;
    return worst ? worst : TW_ERR_INCOMPLETE;
}

#ifdef TW_STATS
int tw_prof_read(tw_ctx* c, unsigned long long* out, size_t cap, int reset) {
    if (!c) return TW_ERR_INVALID;
    return sh_prof_read(c->sh[0], out, cap, reset);
}
#endif

}  // extern "C"
