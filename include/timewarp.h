/*
 * timewarp.h — C ABI of the MI355X batched TimedT emulator (libtimewarp.so).
 *
 * Drop-in boundary for time-warp's pure-emulation path.  The reference has no
 * FFI: its "operator API" is the MonadTimed / MonadTransfer / MonadDialog
 * type-class dictionary, made concrete by the runner
 *     runTimedT :: (MonadIO m, MonadCatch m) => TimedT m a -> m a
 *     (src/Control/TimeWarp/Timed/TimedT.hs:293-304).
 * A scenario written against that API is lowered (host side) into a handler
 * table ("thread programs", the tw_insn ISA below) plus per-link delay/drop
 * tables, and this library runs R independent replicas of it on one GPU.
 * Each entry point names the reference interface it replaces.
 *
 * Conventions: every call returns 0 (TW_OK) or a negative tw_status; nothing
 * throws across the ABI; a tw_ctx is not thread-safe, distinct contexts may be
 * used concurrently from different host threads; device buffers are owned by
 * the library; host buffers passed in are copied before the call returns.
 * There is NO CPU fallback: on a host without a gfx950 device tw_create fails
 * with TW_ERR_NO_DEVICE.
 */
#ifndef TIMEWARP_H
#define TIMEWARP_H

#ifndef __HIPCC_RTC__  /* (the scenario compiler's hiprtc source brings its own types) */
#include <stddef.h>
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 4: the scenario compiler of ABI 3 (tw_set_jit / tw_jit_status /
 * tw_jit_precompile and TW_ERR_JIT) is gone -- measured slower than the
 * interpreter on every configuration.  ABI 3: tw_create(devices,
 * ndev) (was tw_create(device)); the caller-owned reduction buffer of
 * tw_lp_exchange_setup holds TW_LP_RED_WORDS int64 words (was 2).  The scenario
 * descriptor's layout is ABI 2's, but tw_load refuses a descriptor stamped with
 * another version, so a caller built against an older header fails there
 * (TW_ERR_INVALID) instead of handing a red buffer of the old size to the
 * device loop. */
#define TW_ABI_VERSION 4u
#define TW_LP_RED_WORDS 4
/* Async exception payloads (throwTo's value, `SomeException` in the
 * reference's asyncExceptions map, TimedT.hs:113,359) are carried as int64. */

/* ------------------------------------------------------------------ status */
typedef enum tw_status {
    TW_OK = 0,
    TW_ERR_INVALID = -1,      /* malformed descriptor / argument            */
    TW_ERR_NO_DEVICE = -2,    /* no HIP device (or not gfx950)              */
    TW_ERR_HIP = -3,          /* HIP runtime error                          */
    TW_ERR_OOM = -4,          /* device allocation failed                   */
    TW_ERR_STATE = -5,        /* call out of order (run before load, ...)   */
    TW_ERR_REPLICA = -6,      /* one or more replicas ended in error status */
    TW_ERR_INCOMPLETE = -7,   /* tw_run's relaunch cap was reached before every
                                 replica stopped (quiescence / t_end / cap)  */
    TW_ERR_COMM = -8          /* RCCL error (communicator setup or a collective) */
} tw_status;

/* per-replica status (tw_replica_result.status) */
enum {
    TW_REP_RUNNING = 0,       /* queue not empty yet (t_end / event budget) */
    TW_REP_DONE = 1,          /* quiescence: event queue empty (TimedT.hs:239,266-267) */
    TW_REP_ABORTED = 2,       /* an exception escaped runTimedT's loop: async
                                 exception delivered to a forked thread before
                                 its action started (TimedT.hs:252-263, handlers=[]) */
    TW_REP_ERR_SLOTS = 3,     /* thread-slot capacity exceeded              */
    TW_REP_ERR_QUEUE = 4,     /* event-queue capacity exceeded              */
    TW_REP_ERR_FRAMES = 5,    /* catch-frame depth exceeded                 */
    TW_REP_ERR_INSN = 6,      /* bad opcode / pc / link                     */
    TW_REP_ERR_COUNTER = 7    /* the replica's 32-bit insertion counter (seq) or
                                 thread counter (TimedT.hs:288-289) would wrap */
};

/* tie-order probes (tw_tie_audit): events with equal timestamps pop in
 * insertion order (FIFO, the canonical order), reverse insertion order, or a
 * scrambled order.  TimedT orders events by timestamp only (TimedT.hs:100-104),
 * so a replica whose outputs differ between two of these orders depends on
 * pqueue's equal-timestamp order, which no reference test pins. */
enum {
    TW_TIE_FIFO = 0,
    TW_TIE_LIFO = 1,
    TW_TIE_SCRAMBLE = 2,
    TW_TIE_PQUEUE = 3,  /* TimedT's own order: the queue is pqueue-1.3.1.1's
                           binomial MinQueue ordered by timestamp only
                           (TimedT.hs:100-104, 242), throwTo rebuilds it with
                           fromList . map . toList (TimedT.hs:361-368); the
                           wave geometry only (tw_set_tie_mode) */
    TW_TIE_FORKFIRST = 4 /* TW_TIE_FIFO, except that a forked child (fork, a
                           send's deliverer, a delivery's handler, a timeout's
                           watchdog) is always the next pop, ahead of events
                           queued earlier at the same time -- pqueue's rule for
                           an insert whose key is <= the held minimum
                           (TimedT.hs:242, 326-342).  The replica kernels run
                           that child in place, without a queue round trip.
                           Insertion counter values are 31-bit in this mode.
                           Replica geometries but wave (tw_set_tie_mode) */
};

/* ------------------------------------------------------------- exceptions */
/* Exception codes (1..15); handler masks are 16-bit sets over these codes. */
enum {
    TW_EXC_NONE = 0,
    TW_EXC_THREAD_KILLED = 1, /* AsyncException ThreadKilled (killThread, MonadTimed.hs:205-206) */
    TW_EXC_TIMEOUT = 2,       /* MTTimeoutError (MonadTimed.hs:69-73, TimedT.hs:370-376)          */
    TW_EXC_ARITH = 3,         /* ArithException (Overflow etc., ExceptionSpec.hs)                 */
    TW_EXC_USER0 = 4          /* first scenario-defined exception (e.g. ValueReceived)           */
};
#define TW_MASK_ALL 0xFFFEu   /* catchAll: every code 1..15                     */

/* --------------------------------------------------------------------- ISA
 * A thread program is a sequence of tw_insn.  Word w0 = op | a<<8 | b<<16,
 * imm is a signed 32-bit immediate (pc, constant-pool index, value).
 * Registers r0..r3 are int64 per thread; node vars v0..v3 are int64 per node.
 * A thread REF (for throwTo/killThread) is held in a register as
 * slot | (tid << 32) — the engine-specific slot is opaque to programs.
 *
 * Yielding ops end the current step (the reference's ContT capture at `wait`,
 * TimedT.hs:343-355): WAIT_*, FORK (parent waits 1 µs, TimedT.hs:340), SEND
 * (= schedule, i.e. a fork, unless dropped), DELIVER, TMO_BEGIN, END.
 */
enum tw_op {
    TW_OP_NOP = 0,
    TW_OP_END = 1,        /* thread finishes                                      */
    TW_OP_WAIT_REL = 2,   /* wait (for K[imm])    : t = now + K[imm]              */
    TW_OP_WAIT_ABS = 3,   /* wait (till K[imm])   : t = max(now, K[imm])          */
    TW_OP_WAIT_REG = 4,   /* wait (for r[a])      : t = now + max(r[a],0)         */
    TW_OP_FORK = 5,       /* r[a] = ref(child); child pc=imm, regs=copy, node =
                             (b==0xFFFF ? parent node : r[b]); parent waits 1 µs  */
    TW_OP_MYTID = 6,      /* r[a] = ref(self)                                     */
    TW_OP_THROW_TO = 7,   /* throwTo r[a] (code = b&0xFF, value = r[b>>8])        */
    TW_OP_THROW = 8,      /* throwM (code = b&0xFF, value = r[b>>8]) in this thread */
    TW_OP_CATCH = 9,      /* push catch frame: mask = b, handler pc = imm          */
    TW_OP_UNCATCH = 10,   /* pop innermost catch frame (scope left normally)       */
    TW_OP_SETI = 11,      /* r[a] = imm                                           */
    TW_OP_SETK = 12,      /* r[a] = K[imm]                                        */
    TW_OP_ADDI = 13,      /* r[a] += imm                                          */
    TW_OP_MOV = 14,       /* r[a] = r[b]                                          */
    TW_OP_ADD = 15,       /* r[a] += r[b]                                         */
    TW_OP_SUB = 16,       /* r[a] -= r[b]                                         */
    TW_OP_MODI = 17,      /* r[a] = r[a] mod imm (imm > 0, result in [0,imm))     */
    TW_OP_JMP = 18,       /* pc = imm                                             */
    TW_OP_JEQ = 19,       /* if r[a] == r[b&0xFF] pc = imm                        */
    TW_OP_JNE = 20,       /* if r[a] != r[b&0xFF] pc = imm                        */
    TW_OP_JLT = 21,       /* if r[a] <  r[b&0xFF] pc = imm                        */
    TW_OP_JLE = 22,       /* if r[a] <= r[b&0xFF] pc = imm                        */
    TW_OP_JEQI = 23,      /* if r[a] == (int16)b pc = imm                         */
    TW_OP_JNEI = 24,      /* if r[a] != (int16)b pc = imm                         */
    TW_OP_NOW = 25,       /* r[a] = virtualTime (TimedT.hs:322)                   */
    TW_OP_NODE = 26,      /* r[a] = this thread's node                            */
    TW_OP_NLOAD = 27,     /* r[a] = v[node][b]                                    */
    TW_OP_NSTORE = 28,    /* v[node][b] = r[a]                                    */
    TW_OP_LINK = 29,      /* r[a] = out_off[node] + imm  (k-th out-link)          */
    TW_OP_RLINK = 30,     /* r[a] = link_rev[r[b]]       (reply link)             */
    TW_OP_SEND = 31,      /* send over link r[a]: kind = b&0xFF, payload = r[b>>8] */
    TW_OP_DELIVER = 32,   /* (deliver stub) r0=payload r1=link r3=kind            */
    TW_OP_LISTEN = 33,    /* bind this node to listener set imm; b=1: owned by
                             this thread (released when it dies)                 */
    TW_OP_UNLISTEN = 34,  /* unbind this node                                     */
    TW_OP_TRACE = 35,     /* node hash += term(now, 0x30000|imm, r[a])            */
    TW_OP_TMO_BEGIN = 36, /* timeout K[imm] (TimedT.hs:370-376): r[a] = fresh epoch e,
                             done[e] = False, schedule (after K[imm]) watchdog —
                             a fork, so the caller yields 1 µs                   */
    TW_OP_TMO_END = 37,   /* `finally` on normal exit: pop finally frame, done[e]=True */
    TW_OP_TMO_FIRE = 38,  /* (watchdog stub) unless done[r1]: throwTo r0 MTTimeoutError */
    TW_OP_MULI = 39,      /* r[a] *= imm                                          */
    TW_OP_NLOADX = 40,    /* r[a] = v[r[b>>8]][b&0xFF]  (another node's var)      */
    TW_OP_NSTOREX = 41,   /* v[r[b>>8]][b&0xFF] = r[a]                            */
    TW_OP_TMO_PUSH = 42,  /* enter `act `finally` done:=True` for epoch r[a]      */
    TW_OP_COUNT = 43
};

/* Fixed stubs at the start of every program image (validated by tw_load). */
#define TW_PC_DELIVER_STUB 0u  /* WAIT_REG r2 ; DELIVER ; END                   */
#define TW_PC_WATCHDOG_STUB 3u /* WAIT_REG r2 ; TMO_FIRE ; END                  */
#define TW_PC_USER 6u          /* first user instruction                        */
#define TW_PC_NONE 0xFFFFFFFFu
/* listener_pc flag: the handler runs in place in the delivering thread
 * (ForkStrategy `const id`, MonadDialog.hs:114-117) instead of in a thread
 * forked by `fork_` (the default strategy, MonadDialog.hs:317).  The delivering
 * thread takes the handler's registers {payload, link, sender, kind}, moves to
 * the destination node and continues at the handler's pc. */
#define TW_LPC_INLINE 0x80000000u
/* SEND fused with the LINK / RLINK that computes its link (b flags; made by
 * Program.finalize from a `LINK a,k ; SEND a,..` or `RLINK a,r ; SEND a,..`
 * pair, whose SEND stays in the image for jumps to it).  The fused SEND first
 * does what the pair's first instruction does -- VIA_LINK: r[a] = out_off[node]
 * + imm; VIA_RLINK: r[a] = link_rev[r[(b >> 12) & 3]], an out-of-range link
 * stopping the replica as RLINK does -- then sends over r[a] and continues at
 * pc + 2: one instruction (one interpreter pass, one step) instead of two. */
#define TW_SEND_VIA_LINK 0x400u
#define TW_SEND_VIA_RLINK 0x800u
/* Two more pairs fused the same way (the pair's second instruction stays in
 * the image; the fused one continues at pc + 2):
 * TW_ALU_NSTORE (b flag of SETI / SETK / ADDI / MULI / NOW / NODE, whose b is
 *   otherwise unused): `op a,.. ; NSTORE a, var` -- after r[a] is computed,
 *   v[node][b & 3] = r[a];
 * TW_TRACE_PAIR (b flag of TRACE): `TRACE a, tag ; TRACE a2, tag2` -- then
 *   node hash += term(now, 0x30000 | tag2, r[a2]) with a2 = (b >> 13) & 3 and
 *   tag2 = b & 0x1FFF (< 8192). */
#define TW_ALU_NSTORE 0x8000u
#define TW_TRACE_PAIR 0x8000u

typedef struct tw_insn {
    uint32_t w0;  /* op | a<<8 | b<<16 */
    int32_t imm;
} tw_insn;

/* Link-table entry: bits 0..30 delay in µs, bit 31 = drop ("network nastiness").
 * Entry for a send = table[link][ordinal % link_depth][replica], where ordinal
 * counts sends already attempted on that link in that replica (replica-minor,
 * the layout the engine keeps in HBM so lock-stepped lanes coalesce). */
#define TW_LINK_DROP 0x80000000u

/* --------------------------------------------------------------- scenario */
typedef struct tw_scenario_desc {
    uint32_t abi_version;      /* TW_ABI_VERSION */
    uint32_t n_replicas;
    uint32_t n_nodes;
    uint32_t n_insns;
    const tw_insn* insns;
    uint32_t n_consts;
    const int64_t* consts;     /* time constants (µs) and other 64-bit immediates */
    uint32_t main_pc;          /* main thread entry (runs at t=0 without a pop, TimedT.hs:237) */
    uint32_t main_node;
    /* listeners: listener_pc[set * n_msg_kinds + kind] (TW_PC_NONE = no listener) */
    uint32_t n_listener_sets;
    uint32_t n_msg_kinds;
    const uint32_t* listener_pc;
    /* links, CSR over source nodes */
    uint32_t n_links;
    const uint32_t* out_off;   /* n_nodes + 1 */
    const uint32_t* link_dst;  /* n_links */
    const uint32_t* link_rev;  /* n_links (TW_PC_NONE if no reverse link) */
    uint32_t link_depth;       /* >= 1 */
    const uint32_t* link_table;/* [n_links][link_depth][n_replicas]; NULL = all 0 µs */
    const int64_t* node_vars;  /* [n_nodes][4] initial node vars (same for all replicas); NULL = 0 */
    const int64_t* main_regs;  /* [n_replicas][4] initial main-thread registers; NULL = 0 */
    const uint32_t* node_listen; /* [n_nodes] listener set + 1 bound (persistently) at t=0,
                                  0 = unbound; NULL = none (daemons already listening
                                  when the emulation starts) */
    /* capacities (per replica) */
    uint32_t max_slots;        /* concurrent threads                              */
    uint32_t queue_capacity;   /* far-heap entries (live + superseded)           */
    int64_t near_horizon_us;   /* events due within this horizon use the on-chip queue */
    uint32_t max_timeouts;     /* timeout epochs per replica (done-flag bitmap size) */
    uint32_t run_capacity;     /* entries per monotone far-queue run (4 runs per
                                  replica); 0 = far events use the heap only */
    uint32_t max_frames;       /* catch/finally frames per thread (the handler
                                  stack, TimedT.hs:84,198); 0 = 2, at most
                                  TW_MAX_FRAMES.  Two live in the thread record,
                                  deeper ones in a per-slot overflow area.     */
    /* BinaryP wire sizes (Message.hs:155-202): a message of kind k sent over
     * link l is delayed by its transmission time
     * ceil(msg_bytes[k] * 10^6 / link_bw[l]) µs on top of the link-table delay
     * (computed at send time).  NULL / 0 = no transmission time. */
    const uint32_t* msg_bytes; /* [n_msg_kinds] */
    const uint64_t* link_bw;   /* [n_links] bytes per second */
} tw_scenario_desc;

#define TW_MAX_FRAMES 14       /* catch/finally frames per thread (both engines) */

typedef struct tw_replica_result {
    int64_t final_t;           /* curTime after the last pop                     */
    uint64_t events;           /* committed events = PQ.minView pops (TimedT.hs:242) */
    uint64_t delivered;
    uint64_t dropped;          /* link drops                                     */
    uint64_t undeliverable;    /* delivered to an unbound port / unknown kind    */
    uint32_t status;           /* TW_REP_*                                       */
    uint32_t main_exc;         /* uncaught main-thread exception code, rethrown by
                                  runTimedT after quiescence (TimedT.hs:302-304) */
    uint64_t threads;          /* threads ever created (incl. main)              */
    uint32_t tie_flags;        /* tw_tie_audit: bit 0 = audited; bit p = the
                                  outputs under tie probe p (TW_TIE_LIFO,
                                  TW_TIE_SCRAMBLE) differ from the canonical
                                  FIFO order, i.e. the replica depends on the
                                  order of equal-timestamp events            */
    uint32_t reserved;
} tw_replica_result;

typedef struct tw_stats {
    uint64_t events;           /* sum over replicas of this tw_run call          */
    uint64_t sends;            /* delivered + dropped + undeliverable attempts    */
    uint64_t delivered;
    uint64_t dropped;
    uint64_t undeliverable;
    int64_t max_final_t;
    uint32_t replicas_done;
    uint32_t replicas_error;
    uint32_t launches;         /* kernel launches issued by this call            */
    uint32_t reserved;
    double kernel_ms;          /* device time of the event kernels (HIP events)  */
    double wall_ms;            /* host wall time of the call                     */
} tw_stats;

typedef struct tw_ctx tw_ctx;

/* Create a context over `ndev` HIP devices of this process, devices[0..ndev)
 * (no CPU fallback; each must be a gfx950).  SURVEY.md 8(b)'s runner over a
 * node's GPUs: with ndev > 1 the library owns one RCCL communicator per
 * device (ncclCommInitAll) --
 *   tw_load / tw_lpb_load split the replicas into contiguous blocks
 *     [g*R/G, (g+1)*R/G); tw_run runs every block at once
 *     and all-reduces the statistics over RCCL; results and hashes read back
 *     in replica order;
 *   tw_lp_load splits the node range; tw_lp_run runs the window loop with the
 *     record blocks moved by RCCL send/recv and the window words by RCCL
 *     all-reduce(min).
 * A device listed more than once (or TW_TRANSPORT=copy) moves the blocks and
 * words by device copies ordered with HIP events instead (same results).
 * Replaces runTimedT (TimedT.hs:293-304) for a batch spread over GPUs. */
int tw_create(const int* devices, int ndev, tw_ctx** out);

/* One process per GPU (e.g. torchrun): rank 0 makes a job id with
 * tw_comm_id, the caller hands it to every rank (any side channel), and each
 * rank calls tw_create_rank; the library then owns an RCCL communicator over
 * the ranks (ncclCommInitRank).  tw_load takes this rank's block of replicas;
 * tw_run's stats and tw_lp_results are the whole job's; tw_lp_run exchanges
 * with the other ranks itself.  nranks == 1 is a one-rank job (its
 * collectives still go through RCCL). */
#define TW_COMM_ID_BYTES 128
int tw_comm_id(uint8_t id[TW_COMM_ID_BYTES]);
int tw_create_rank(int device, int nranks, int rank, const uint8_t id[TW_COMM_ID_BYTES], tw_ctx** out);
/* Shape of a context: devices of this process, ranks of the job, the global
 * rank of its first device, transport (0 none, 1 RCCL, 2 device copies). */
int tw_ctx_info(tw_ctx* ctx, int* ndev, int* world, int* rank0, int* transport);

/* Copy a lowered scenario into HBM and reset every replica to t=0, queue empty,
 * main thread about to run (TimedT.hs:120-127, 234-237).  Replaces the
 * construction of the TimedT value + emptyScenario. */
int tw_load(tw_ctx* ctx, const tw_scenario_desc* desc);

/* Reset every replica of the loaded scenario to its initial state (t=0, main
 * about to run) without re-uploading tables: the device-resident equivalent of
 * evaluating runTimedT again on the same scenario.  Stream-ordered, async. */
int tw_reset(tw_ctx* ctx);

/* Run every replica's event loop (launchTimedT, TimedT.hs:234-286) until its
 * queue is empty, the next event is later than t_end_us, or its committed-event
 * total (since tw_load) reached max_events (UINT64_MAX = no cap).  May be called
 * repeatedly to advance in pieces.  Blocking.  Replaces runTimedT.  `out` is
 * the whole job's (every device, every rank: counts summed, times the max). */
int tw_run(tw_ctx* ctx, int64_t t_end_us, uint64_t max_events, tw_stats* out);

/* Per-replica results (final virtual time, counters, status, main exception). */
int tw_read_results(tw_ctx* ctx, tw_replica_result* out, size_t n_replicas);

/* Per-node trace hashes, layout [replica][node] (n = n_replicas * n_nodes). */
int tw_read_hashes(tw_ctx* ctx, uint64_t* out, size_t n);

/* Convenience aggregate of tw_read_results. */
int tw_read_final(tw_ctx* ctx, int64_t* max_final_t, uint64_t* delivered,
                  uint64_t* dropped, uint64_t* events);

/* Trace records: every executed TRACE instruction (the reference's
 * `logMeasure` / log lines, bench/Network/Common/Bench/Network/Commons.hs:
 * 121-171 and Sender/Main.hs:46-61, Receiver/Main.hs:33-38) appended to a
 * per-replica buffer, in the replica's execution order: the input of the
 * LogReader's measures.csv (bench/Network/LogReader/Main.hs:85-119). */
typedef struct tw_trace_rec {
    int64_t t;      /* virtual time (µs)                    */
    int64_t val;    /* the traced register                  */
    uint32_t node;  /* the running thread's node            */
    uint32_t tag;   /* the TRACE immediate                  */
} tw_trace_rec;

/* Record up to cap TRACE records per replica from the next tw_reset on
 * (0 = off, the default; the count beyond cap is still reported).  Call after
 * tw_load; allocates cap * n_replicas * 32 bytes of HBM. */
int tw_set_trace(tw_ctx* ctx, uint32_t cap);

/* A replica's trace records: copies min(cap, emitted, trace cap) records and
 * stores the number emitted (possibly more than were kept) in *n_emitted. */
int tw_read_trace(tw_ctx* ctx, uint32_t replica, tw_trace_rec* out, size_t cap, uint64_t* n_emitted);

/* Tie-order audit: run every replica (as tw_run with t_end_us / max_events)
 * under each probe order p in 1..probes (TW_TIE_LIFO, TW_TIE_SCRAMBLE), then
 * under the canonical order, and set tie_flags bit p of every replica whose
 * results or node
 * hashes differ from the canonical run's.  The canonical run's state is left
 * loaded, so results/hashes read afterwards are the canonical ones.  `out`
 * gets the canonical run's stats.  Replaces nothing in the reference: it
 * flags the replicas for which TimedT's pqueue tie order (TimedT.hs:100-104,
 * 242) could give a different trace than this engine. */
int tw_tie_audit(tw_ctx* ctx, int64_t t_end_us, uint64_t max_events, uint32_t probes, tw_stats* out);

/* The equal-timestamp order of later tw_reset / tw_run calls: TW_TIE_FIFO
 * (the default, the engine's (t, seq) order), TW_TIE_LIFO / TW_TIE_SCRAMBLE
 * (the audit probes), or TW_TIE_PQUEUE: TimedT's structural order, so a replica
 * tw_tie_audit flagged can be re-run exactly as TimedT orders it (pqueue's
 * MinQueue, PARITY UNPINNED against pqueue itself: its sources are not in the
 * reference; equal to the oracle's pqueue transcription).  PQUEUE needs the
 * wave geometry (TW_ERR_INVALID otherwise) and a queue_capacity covering the
 * replica's pending events. */
int tw_set_tie_mode(tw_ctx* ctx, uint32_t mode);

/* Testing hook: from the next tw_reset on, start every replica's insertion
 * counter at seq0 and its thread counter at tid0 (>= 1; main is tid 0), so the
 * TW_REP_ERR_COUNTER guard can be reached in a short run. */
int tw_set_counter_base(tw_ctx* ctx, uint32_t seq0, uint32_t tid0);

/* Kernel geometry of the loaded scenario, chosen by tw_load from the replica
 * count (environment TW_GEOMETRY=dense|sparse|half|wave|narrow|compact overrides):
 *   DENSE  one lane per replica, 256 replicas per workgroup (many replicas);
 *   SPARSE one lane per replica, 16 per workgroup, large on-chip queue;
 *   HALF   the dense layout as two 32-lane waves per SIMD (an experiment);
 *   WAVE   one wavefront per replica: lane-parallel queue (few replicas);
 *   NARROW the dense layout with one 64-replica wave per workgroup (fewer
 *          replicas than fill the GPU: the waves spread over every CU);
 *   LP     node-partitioned mode (tw_lp_load);
 *   LPB    batched node-partitioned mode (tw_lpb_load);
 *   COMPACT the dense layout without far runs (far events in the HBM heap
 *          only) and an 8-entry on-chip queue, two waves per SIMD: dense
 *          batches of scenarios with run_capacity 0 (TW_GEOMETRY=compact). */
enum { TW_GEO_DENSE = 0, TW_GEO_SPARSE = 1, TW_GEO_HALF = 2, TW_GEO_WAVE = 3, TW_GEO_LP = 4, TW_GEO_NARROW = 5,
       TW_GEO_LPB = 6, TW_GEO_COMPACT = 7 };
int tw_geometry(tw_ctx* ctx);

/* Duration (ms) of every event-kernel launch of the last tw_run, measured with
 * HIP events on the library's stream; returns the count written. */
int tw_last_launch_ms(tw_ctx* ctx, double* out, size_t cap);

void tw_destroy(tw_ctx* ctx);
const char* tw_strerror(int code);
const char* tw_version(void);

/* ---------------------------------------------- link tables drawn on the GPU
 * The scenario builders' network-delay draws (examples/token-ring/Main.hs:60,77:
 * `mkStdGen` + `getRandomTR`, random-1.1's StdGen) for every replica at once:
 * replica r's generator is mkStdGen(seed_base + r); it walks the links with
 * drawn[l] != 0 in ascending order and, for each, draws link_depth entries,
 * each randomR(lo[l], hi[l]) followed -- when drop_log2 > 0 -- by a drop coin
 * randomR(0, 2^drop_log2 - 1) that marks the entry TW_LINK_DROP when 0.  Links
 * with drawn[l] == 0 hold lo[l] in every entry.  Output: the table tw_load
 * takes, [n_links][link_depth][n_replicas] in host memory, equal entry for
 * entry to the host draw (time-warp_amd/timewarp/stdgen.py); one GPU thread
 * per replica replaces a host loop of n_links x link_depth vector steps.
 * Ranges must need one StdGen digit (hi - lo + 1 <= 2147483). */
typedef struct tw_table_draw {
    uint32_t n_links;
    uint32_t link_depth;
    uint32_t n_replicas;
    int32_t drop_log2;         /* 0 = no drop coins, else 1..21 (one digit) */
    int64_t seed_base;
    const uint8_t* drawn;      /* [n_links] */
    const int64_t* lo;         /* [n_links] µs */
    const int64_t* hi;         /* [n_links] µs (drawn links) */
} tw_table_draw;
int tw_draw_link_table(int device, const tw_table_draw* spec, uint32_t* out);

/* ------------------------------------------------- node-partitioned (LP) mode
 * One huge scenario (n_replicas = 1) split by node across contexts / GPUs
 * (BASELINE config 4).  Each lane runs one node as a logical process with its
 * own queue; a send whose delay is >= the lookahead becomes a delivery record
 * for the destination node, and time advances in conservative windows
 * [T, T + lookahead) with T = the minimum next-event time over all contexts.
 * Counts and trace hashes equal a sequential TimedT run of the same scenario
 * for any scenario whose outputs do not depend on equal-timestamp order (the
 * oracle's tie audit); the deliverer thread's three pops (TimedT.hs:339-355 via
 * `schedule`) are accounted at the sender (start, wake) and at the receiver
 * (resume after the handler fork). */
typedef struct tw_lp_record {
    int64_t t_arr;     /* delivery time (send time + link delay)         */
    int64_t payload;
    uint32_t link;
    uint32_t kind;
    uint32_t src;      /* sending node                                   */
    uint32_t dst;      /* receiving node (global id)                     */
} tw_lp_record;

/* Load the whole scenario (desc->n_replicas must be 1) and own nodes
 * [lp_begin, lp_begin + lp_count).  lookahead_us must not exceed any link delay
 * (a shorter send is a TW_REP_ERR_INSN status).  Replaces runTimedT for one
 * scenario partitioned by node. */
int tw_lp_load(tw_ctx* ctx, const tw_scenario_desc* desc, uint32_t lp_begin, uint32_t lp_count,
               int64_t lookahead_us, uint32_t inbox_cap, uint32_t outbox_cap);
/* Process every local event with t < t_end_excl; deliver records addressed to
 * local nodes; *next_t = earliest pending local event (INT64_MAX if none);
 * *n_foreign = records waiting for tw_lp_take_outbox. */
int tw_lp_window(tw_ctx* ctx, int64_t t_end_excl, int64_t* next_t, uint64_t* n_foreign);
/* Move the foreign records out (host buffer), for an exchange (RCCL all-to-all). */
int tw_lp_take_outbox(tw_ctx* ctx, tw_lp_record* out, size_t cap, size_t* n);
/* Hand records addressed to local nodes in; updates *next_t. */
int tw_lp_inject(tw_ctx* ctx, const tw_lp_record* recs, size_t n, int64_t* next_t);
/* Aggregate counters (final_t = max, counts = sums, status = worst) and node
 * hash additions (length n_nodes; a scenario's hashes are the sum over
 * contexts mod 2^64).  A one-device context without a communicator reports
 * its own nodes; a multi-device or RCCL context the whole job's (reduced
 * over its devices and ranks). */
int tw_lp_results(tw_ctx* ctx, tw_replica_result* agg, uint64_t* node_hashes, size_t n_nodes);

/* ---- batched node-partitioned mode (intra-replica parallelism)
 * R replicas of a scenario whose nodes interact only through sends of at
 * least lookahead_us (plus forks onto other nodes issued before any node runs
 * past the fork time, e.g. a main thread that starts the node daemons):
 * every (node, replica) pair is a lane, a logical process with its own queue,
 * and the replicas share one device-driven window loop.  A replica's events
 * then run in parallel across its nodes instead of in one sequential chain
 * (a hotspot receiver's backlog is sorted per window by tw_lp_due instead of
 * being queued).  After tw_lpb_load the replica API applies unchanged:
 * tw_reset, tw_run (t_end_us = INT64_MAX, max_events = UINT64_MAX only: the
 * whole window loop), tw_read_results / tw_read_hashes per replica, with
 * results equal to runTimedT's (TimedT.hs:293-304) for scenarios whose outputs
 * do not depend on equal-timestamp order (the oracle's tie audit).  The
 * replica count must be a power of two; node_inbox_cap[n] (NULL: inbox_cap
 * for every node, each <= 2048) bounds the delivery records pending at node n
 * of one replica; outbox_cap bounds the records of one tick.  A fork's ref to
 * a child on another node is opaque (-1). */
int tw_lpb_load(tw_ctx* ctx, const tw_scenario_desc* desc, int64_t lookahead_us, const uint32_t* node_inbox_cap,
                uint32_t inbox_cap, uint32_t outbox_cap);
/* Windows and ticks of the last tw_run in batched mode. */
int tw_lpb_windows(tw_ctx* ctx, uint64_t* windows, uint64_t* ticks);
/* Batched mode, since the last tw_reset: the due records (the delivery records
 * of heavy nodes, sorted per window) and how many of them ran data-parallel --
 * one per thread, ahead of the node's own chain -- because their handler is
 * batchable (the fork_-dispatched handler of a (listener set, kind) whose
 * effects are its own: registers, node-variable reads, links, traces, at most
 * one send followed by END; bench/Network's Ping handler) and no other event of
 * the node falls between their events.  Results are those of the sequential
 * loop either way; TW_LP_BATCH=0 at tw_lpb_load turns the batch off. */
int tw_lpb_batch(tw_ctx* ctx, uint64_t* batched, uint64_t* due_records);

/* ---- device-driven windows (no host round trip per window)
 * The window loop above costs several host synchronisations per window.  Here
 * the device keeps the window start T, the work lists and the window count,
 * and advances T itself.  One "tick" is: the event kernel over window
 * [T, T + lookahead), the local delivery of this context's records, and the
 * packing of foreign records into fixed per-rank blocks; then, between
 * ranks, an all-to-all of those blocks and an all-reduce(min) of four int64
 * words; then the advance: when no rank has work left in the window, T := the
 * global next-event time (INT64_MAX: done), else the same window runs again.
 * Records are drained into node queues only at a window's first tick, so the
 * result does not depend on how many ticks a window took.  Every kernel goes
 * on the context's stream (tw_set_stream: the caller's, e.g. the stream its
 * RCCL collectives run on), so a caller enqueues many ticks and synchronises
 * once (tw_lp_progress).  Replaces the MonadDialog send path's cross-node hop
 * (MonadDialog.hs:149-166) with an on-device exchange.
 *
 * Block layout (send and recv, world blocks of (cap + 1) tw_lp_records):
 * record 0 of block g is a header whose first uint32 is the record count, then
 * up to cap records (the header counts every record meant for that rank: the
 * ones beyond cap wait in a carry buffer for the next tick, whose window then
 * reruns -- never an overflow).  red: 4 device int64 {next event time,
 * -(lanes active), -(overflow bits), -(largest per-rank record count)},
 * all-reduced with MIN between tw_lp_tick_import and tw_lp_tick_end: an
 * overflow on any rank (tw_lp_state.err) ends every rank's loop at the same
 * tick, with bit 16 set. */
typedef struct tw_lp_state {
    uint64_t windows;   /* windows completed                                 */
    uint64_t ticks;     /* ticks run (>= windows)                            */
    int64_t  t;         /* current window start (INT64_MAX when done)        */
    uint32_t done;      /* 1: every queue is empty everywhere                */
    uint32_t err;       /* inbox / outbox / exchange-block overflow bits; bit
                           16: the loop stopped because some rank overflowed */
} tw_lp_state;
/* Use the caller's HIP stream (hipStream_t) for every later call; NULL = the
 * context's own stream. */
int tw_set_stream(tw_ctx* ctx, void* hip_stream);
/* world == 1: send/recv/red may be NULL (the context keeps its own red).
 * starts: host array of world + 1 node boundaries (rank g owns nodes
 * [starts[g], starts[g+1])).  send/recv: device buffers of
 * world * (cap + 1) * 32 bytes; red: device int64[TW_LP_RED_WORDS]. */
int tw_lp_exchange_setup(tw_ctx* ctx, uint32_t world, uint32_t rank, const uint32_t* starts, void* send,
                         void* recv, uint32_t cap, int64_t* red);
/* Start the device loop at T = 0 (after tw_reset). */
int tw_lp_loop_begin(tw_ctx* ctx);
/* Enqueue a tick's first half: event kernel + local delivery + packing. */
int tw_lp_tick(tw_ctx* ctx);
/* After the all-to-all: deliver recv's records; fill red. */
int tw_lp_tick_import(tw_ctx* ctx);
/* After the all-reduce of red: advance the window or rerun it. */
int tw_lp_tick_end(tw_ctx* ctx);
/* Synchronise the stream once and read the loop's state. */
int tw_lp_progress(tw_ctx* ctx, tw_lp_state* out);
/* Single context (world 1): enqueue ticks in batches of 16 with one host
 * synchronisation per batch until done or max_ticks. */
int tw_lp_run_windows(tw_ctx* ctx, uint64_t max_ticks, tw_lp_state* out);
/* The whole device window loop from t = 0 (after tw_reset) over every device
 * and rank of the context, the exchange owned by the library: per tick the
 * event kernels and packing, the record blocks between ranks (RCCL
 * send/recv), the import, an RCCL all-reduce(min) of the window words, the
 * advance; one host synchronisation per 16 ticks.  Blocks travel at the size
 * the ranks last agreed on -- the largest per-rank demand of a tick, rounded
 * up, re-chosen every 16 ticks from the reduced words (TW_LP_XCAP caps it,
 * default 16384 records); records beyond it wait a tick in a carry buffer
 * (the window reruns) and go first at the next tick.  The carry holds up to
 * min(outbox capacity, 2^20) records: a demand above the agreed block size
 * for long enough to outgrow it stops every rank at the same tick with the
 * replica error (tw_lp_state.err bit 8) rather than losing a record.  A local
 * failure on one rank is agreed over the job before the next collective, so
 * every rank returns the same code at the same point -- a failure the shard
 * can still report: after a HIP fault that leaves the device unusable (a
 * kernel fault, a lost device), that rank's next RCCL call fails or never
 * completes, and the ranks waiting in the collective with it stay stranded
 * until RCCL's own timeout; nothing in the library can end them sooner.  A
 * context whose RCCL call failed is marked unusable: every later call that
 * communicates (tw_run, tw_tie_audit, tw_lp_run, tw_lp_results) returns
 * TW_ERR_COMM at once, without entering a collective; tw_destroy it and make
 * a new one.  The multi-GPU
 * replacement of MonadDialog's cross-node send path (MonadDialog.hs:149-166)
 * with runTimedT's loop around it.  The caller-driven primitives
 * (tw_lp_exchange_setup / tw_lp_tick ...) remain for one-device contexts. */
int tw_lp_run(tw_ctx* ctx, uint64_t max_ticks, tw_lp_state* out);

/* ---------------------------------------------------------------- hashing
 * Per-node trace hash (made fully commutative): every
 * committed event / trace / delivery at node n adds term(t, kind, val) to
 * H[n] modulo 2^64.  Thread ids never enter a term (they depend on global pop
 * order, TimedT.hs:288-289).  Shared by the engine and the oracle. */
static inline uint64_t tw_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
/* (t, kind) packs injectively into 64 bits for t < 2^44 µs (~203 days) and
 * kind < 2^20; val enters through its own mix (mix64(0) = 0). */
static inline uint64_t tw_term(int64_t t, uint32_t kind, int64_t val) {
    uint64_t v = val ? tw_mix64((uint64_t)val ^ 0x9e3779b97f4a7c15ull) : 0ull;
    return tw_mix64((((uint64_t)t << 20) | kind) ^ v);
}
#define TW_KIND_RESUME 0x10000u   /* | pc        : a thread resumed at pc       */
#define TW_KIND_EXC 0x20000u      /* | exc code  : async exception delivered    */
#define TW_KIND_TRACE 0x30000u    /* | tag       : explicit TRACE               */
#define TW_KIND_RECV 0x40000u     /* | msg kind  : message delivered to node    */
#define TW_KIND_DROP 0x50000u     /* | msg kind  : link dropped the message     */
#define TW_KIND_UNDELIV 0x60000u  /* | msg kind  : no listener at destination   */

#ifdef __cplusplus
}
#endif
#endif /* TIMEWARP_H */
