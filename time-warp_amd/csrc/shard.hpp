// shard.hpp — one device's engine context (engine.hip) as seen by the public
// C ABI (abi.hip).  A tw_ctx (include/timewarp.h) holds one shard per device
// of this process; each shard is the single-device engine of rounds 1-2: one
// HIP device, one stream, its replicas (or logical processes) in HBM.  These
// entry points are internal to libtimewarp.so (hidden symbols).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/timewarp.h"

struct tw_shard;

namespace tw {

#define TW_HIDDEN __attribute__((visibility("hidden")))

TW_HIDDEN int sh_create(int device, tw_shard** out);
TW_HIDDEN void sh_destroy(tw_shard* c);
TW_HIDDEN int sh_load(tw_shard* c, const tw_scenario_desc* s);
TW_HIDDEN int sh_lp_load(tw_shard* c, const tw_scenario_desc* s, uint32_t lp_begin, uint32_t lp_count,
                         int64_t lookahead_us, uint32_t inbox_cap, uint32_t outbox_cap);
TW_HIDDEN int sh_lpb_load(tw_shard* c, const tw_scenario_desc* s, int64_t lookahead_us, const uint32_t* node_inbox_cap,
                          uint32_t inbox_cap, uint32_t outbox_cap);
TW_HIDDEN int sh_reset(tw_shard* c);
TW_HIDDEN int sh_run(tw_shard* c, int64_t t_end_us, uint64_t max_events, tw_stats* out);
TW_HIDDEN int sh_read_results(tw_shard* c, tw_replica_result* out, size_t n);
TW_HIDDEN int sh_read_hashes(tw_shard* c, uint64_t* out, size_t n);
TW_HIDDEN int sh_tie_audit(tw_shard* c, int64_t t_end_us, uint64_t max_events, uint32_t probes, tw_stats* out);
TW_HIDDEN int sh_geometry(tw_shard* c);
TW_HIDDEN int sh_set_counter_base(tw_shard* c, uint32_t seq0, uint32_t tid0);
TW_HIDDEN int sh_set_tie_mode(tw_shard* c, uint32_t mode);
TW_HIDDEN int sh_set_trace(tw_shard* c, uint32_t cap);
TW_HIDDEN int sh_read_trace(tw_shard* c, uint32_t replica, tw_trace_rec* out, size_t cap, uint64_t* n_emitted);
TW_HIDDEN int sh_last_launch_ms(tw_shard* c, double* out, size_t cap);
TW_HIDDEN int sh_prof_read(tw_shard* c, unsigned long long* out, size_t cap, int reset);
// shape of what a shard holds: replicas its results cover (batched LP: the
// replica count, not the lanes), nodes per replica, LP node range
TW_HIDDEN uint32_t sh_replicas(tw_shard* c);
TW_HIDDEN uint32_t sh_nodes(tw_shard* c);
TW_HIDDEN bool sh_is_lp(tw_shard* c);
TW_HIDDEN int sh_device(tw_shard* c);

// node-partitioned (LP) mode
TW_HIDDEN int sh_lp_window(tw_shard* c, int64_t t_end_excl, int64_t* next_t, uint64_t* n_foreign);
TW_HIDDEN int sh_lp_take_outbox(tw_shard* c, tw_lp_record* out, size_t cap, size_t* n);
TW_HIDDEN int sh_lp_inject(tw_shard* c, const tw_lp_record* recs, size_t n, int64_t* next_t);
TW_HIDDEN int sh_lp_results(tw_shard* c, tw_replica_result* agg, uint64_t* node_hashes, size_t n_nodes);
TW_HIDDEN int sh_lpb_windows(tw_shard* c, uint64_t* windows, uint64_t* ticks);
TW_HIDDEN int sh_lpb_batch(tw_shard* c, uint64_t* batched, uint64_t* due);
TW_HIDDEN int sh_set_stream(tw_shard* c, void* hip_stream);
TW_HIDDEN int sh_lp_exchange_setup(tw_shard* c, uint32_t world, uint32_t rank, const uint32_t* starts, void* send,
                                   void* recv, uint32_t cap, int64_t* red);
TW_HIDDEN int sh_lp_loop_begin(tw_shard* c);
TW_HIDDEN int sh_lp_tick(tw_shard* c);
TW_HIDDEN int sh_lp_tick_import(tw_shard* c);
TW_HIDDEN int sh_lp_tick_end(tw_shard* c);
TW_HIDDEN int sh_lp_progress(tw_shard* c, tw_lp_state* out);
TW_HIDDEN int sh_lp_run_windows(tw_shard* c, uint64_t max_ticks, tw_lp_state* out);

// the library-driven exchange (abi.hip): library-owned blocks of `cap`
// records per rank, of which the first cap_eff travel each tick
struct ShardXchg {
    int device;
    hipStream_t stream;
    void* send;       // world blocks of (stride + 1) x 32 B: header + records
    void* recv;
    int64_t* red;     // RD_COUNT words, all-reduced with MIN
    uint32_t world, stride, cap_eff;
};
TW_HIDDEN int sh_lp_exchange_own(tw_shard* c, uint32_t world, uint32_t rank, const uint32_t* starts, uint32_t cap);
TW_HIDDEN void sh_lp_exchange_info(tw_shard* c, ShardXchg* x);
TW_HIDDEN int sh_lp_set_block(tw_shard* c, uint32_t cap_eff);
TW_HIDDEN int64_t sh_lp_xmax(tw_shard* c);
TW_HIDDEN int sh_lp_clear_xmax(tw_shard* c);

}  // namespace tw
