// oracle/timedt_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of time-warp's pure-emulation runner, used as the parity
// checker for the HIP engine and as the timed CPU baseline ("port").  Only
// tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
// The product path (libtimewarp.so) never links or calls this file.
//
// What it restates (file:line in /root/reference):
//   Scenario state        src/Control/TimeWarp/Timed/TimedT.hs:107-127
//   event loop            TimedT.hs:234-286 (pop min, curTime := t, take async
//                         exception for tid, raise it or run the continuation
//                         under the thread's handler stack)
//   runTimedT             TimedT.hs:293-304 (main's exception rethrown after
//                         quiescence)
//   fork                  TimedT.hs:326-342 (tid = counter++, child queued at
//                         now with handlers [], parent `wait (for 1 mcs)`)
//   wait                  TimedT.hs:343-355 (queue at max cur (rel cur))
//   throwTo/wakeUpThread  TimedT.hs:357-368 (events of tid re-stamped to now by
//                         `PQ.fromList . map f . PQ.toList`; first exception wins)
//   timeout               TimedT.hs:370-376 (schedule (after t) watchdog;
//                         act `finally` done := True)
//   catch / handler stack TimedT.hs:183-204, 263, 284
//   schedule/invoke/...   MonadTimed.hs:162-206
// plus the build-defined emulated transfer of SURVEY.md Appendix A.3 (the
// reference's PureRpc is absent; its usage: examples/token-ring/Main.hs:73-85).
//
// Two queue modes:
//   mode 0 "canonical": events ordered by (t, seq), seq = per-run insertion
//          counter; throwTo gives the target's event (now, fresh seq).  This is
//          the order the GPU engine implements bit-exactly.
//   mode 1 "pqueue":    pqueue-1.3.1.1 MinQueue transcription (pqueue_min.hpp),
//          ordered by timestamp only, throwTo rebuilds the whole queue exactly
//          as TimedT.hs:368.  Used for the tie-order audit (parity unpinned).
//   modes 2, 3: the canonical queue with equal timestamps in reverse insertion
//          order (TW_TIE_LIFO) or a scrambled order (TW_TIE_SCRAMBLE): the
//          engine's tie probes (tw_tie_audit), mirrored for the parity tests.
//   mode 5: the canonical queue, but a forked child is always the next pop
//          (TW_TIE_FORKFIRST): its entry takes the key of its insertion counter
//          value alone, every other entry the value with bit 31 set, so it
//          sorts before everything queued at the same time -- what pqueue's
//          MinQueue does with an insert whose key is <= the held minimum.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <thread>
#include <vector>

#include "../include/timewarp.h"
#include "pqueue_min.hpp"
#include "stdgen.hpp"

extern "C" {

// Live delay specification (the reference's `Delays` function evaluated with a
// live StdGen in pop order, examples/token-ring/Main.hs:73-77).  Used for the
// CPU-only config and to record link tables for the GPU (record-replay).
typedef struct two_live_delays {
    const uint32_t* kind;   // per link: 0 = use desc table, 1 = constant lo, 2 = U[lo,hi] draw
    const int64_t* lo;      // per link
    const int64_t* hi;      // per link
    int64_t seed;           // mkStdGen seed for this replica's generator
    uint32_t* record;       // optional [n_links][record_depth] recorded entries
    uint32_t record_depth;
    uint32_t record_overflow;  // out: set if an ordinal >= record_depth was drawn
} two_live_delays;

typedef struct two_term {
    int64_t t;
    uint32_t node;
    uint32_t kind;
    int64_t val;
} two_term;

typedef struct two_opts {
    int mode;                // 0 canonical, 1 pqueue
    int64_t t_end;           // stop before popping an event later than this
    uint64_t max_events;     // 0 = unlimited
    two_live_delays* live;   // optional
    two_term* terms;         // optional log of every hash term
    size_t terms_cap;
    size_t terms_n;          // out
    two_term* traces;        // optional log of TRACE terms only
    size_t traces_cap;
    size_t traces_n;         // out
} two_opts;

}  // extern "C"

namespace {

constexpr uint32_t kStepCap = 1u << 22;  // instructions per step before TW_REP_ERR_INSN

struct Frame {
    uint16_t mask;  // 0 => finally frame of timeout epoch `pc`
    uint16_t pc;
};

struct Thread {
    uint64_t tid = 0;
    uint32_t node = 0;
    uint32_t pc = 0;
    int64_t r[4] = {0, 0, 0, 0};
    Frame fr[TW_MAX_FRAMES];  // the handler list (TimedT.hs:84,198), innermost last
    int nfr = 0;
    bool started = false;
    bool is_main = false;
    bool alive = true;
    int64_t hpos = -1;  // canonical heap position (-1: no queued event)
};

struct Event {
    int64_t t;
    uint64_t seq;
    Thread* th;
};

struct Exc {
    uint32_t code;
    int64_t val;
};

struct EvLEq {  // Event's Ord: compare timestamps only (TimedT.hs:100-104)
    bool operator()(const Event& a, const Event& b) const { return a.t <= b.t; }
};

// The key an insertion counter takes under a tie mode (== the engine's seq_key).
// (TW_TIE_FORKFIRST: a forked child's entry is marked by bit 40 of its seq and
// keeps the bare value, CanonQueue::key)
constexpr uint64_t kChildMark = 1ull << 40;
inline uint32_t seq_key32(int tie, uint32_t s) {
    if (tie == TW_TIE_FIFO) return s;
    if (tie == TW_TIE_FORKFIRST) return s | 0x80000000u;
    if (tie == TW_TIE_LIFO) return 0u - s;
    uint32_t x = s;
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// Canonical (t, seq) binary heap with thread back-pointers for re-stamping.
// Equal timestamps pop in the order of seq_key32(tie, seq).
class CanonQueue {
  public:
    int tie = TW_TIE_FIFO;
    bool empty() const { return h_.empty(); }
    size_t size() const { return h_.size(); }
    void insert(const Event& e) {
        h_.push_back(e);
        e.th->hpos = (int64_t)h_.size() - 1;
        up(h_.size() - 1);
    }
    Event pop() {
        Event top = h_[0];
        top.th->hpos = -1;
        Event last = h_.back();
        h_.pop_back();
        if (!h_.empty()) {
            h_[0] = last;
            last.th->hpos = 0;
            down(0);
        }
        return top;
    }
    void restamp(Thread* th, int64_t t, uint64_t seq) {  // decrease-key to (now, fresh seq)
        size_t i = (size_t)th->hpos;
        h_[i].t = t;
        h_[i].seq = seq;
        up(i);
        down((size_t)th->hpos);
    }

  private:
    uint32_t key(const Event& e) const {
        if (tie == TW_TIE_FORKFIRST && (e.seq & kChildMark)) return (uint32_t)e.seq;
        return seq_key32(tie, (uint32_t)e.seq);
    }
    bool less(const Event& a, const Event& b) const {
        if (a.t != b.t) return a.t < b.t;
        if (tie == TW_TIE_FIFO) return a.seq < b.seq;
        return key(a) < key(b);
    }
    void set(size_t i, const Event& e) {
        h_[i] = e;
        e.th->hpos = (int64_t)i;
    }
    void up(size_t i) {
        Event e = h_[i];
        while (i > 0) {
            size_t p = (i - 1) / 2;
            if (!less(e, h_[p])) break;
            set(i, h_[p]);
            i = p;
        }
        set(i, e);
    }
    void down(size_t i) {
        Event e = h_[i];
        size_t n = h_.size();
        for (;;) {
            size_t c = 2 * i + 1;
            if (c >= n) break;
            if (c + 1 < n && less(h_[c + 1], h_[c])) ++c;
            if (!less(h_[c], e)) break;
            set(i, h_[c]);
            i = c;
        }
        set(i, e);
    }
    std::vector<Event> h_;
};

struct Sim {
    const tw_scenario_desc* d;
    uint32_t replica;
    two_opts* o;
    int mode;

    // Scenario (TimedT.hs:107-127)
    CanonQueue cq;
    PQueueMin<Event, EvLEq> pq;
    int64_t cur = 0;
    std::map<uint64_t, Exc> async_exc;  // keyed by thread id, like TimedT.hs:113
    uint64_t threads_counter = 0;
    uint64_t seq = 0;

    std::vector<std::unique_ptr<Thread>> by_tid;  // index = tid; freed once dead
    std::vector<int64_t> node_vars;   // [node][4]
    std::vector<uint32_t> bind;       // 0 = unbound, else set+1
    std::vector<uint64_t> bind_owner; // tid or UINT64_MAX (persistent)
    std::vector<uint32_t> link_ord;
    std::vector<uint8_t> tmo_done;
    uint32_t tmo_ctr = 0;
    StdGen gen{1, 1};

    uint64_t* hashes;
    tw_replica_result res{};
    uint64_t live_slots = 0;  // concurrent threads, checked against max_slots

    uint32_t max_frames;

    Sim(const tw_scenario_desc* d_, uint32_t rep, two_opts* o_, uint64_t* hashes_)
        : d(d_), replica(rep), o(o_), mode(o_->mode == 1 ? 1 : 0), hashes(hashes_) {
        cq.tie = o_->mode == 5 ? TW_TIE_FORKFIRST : o_->mode >= 2 ? o_->mode - 1 : TW_TIE_FIFO;
        max_frames = d->max_frames ? d->max_frames : 2u;
        node_vars.assign((size_t)d->n_nodes * 4, 0);
        if (d->node_vars) std::memcpy(node_vars.data(), d->node_vars, node_vars.size() * 8);
        bind.assign(d->n_nodes, 0);
        bind_owner.assign(d->n_nodes, UINT64_MAX);
        if (d->node_listen)
            for (uint32_t n = 0; n < d->n_nodes; ++n) bind[n] = d->node_listen[n];
        link_ord.assign(d->n_links, 0);
        tmo_done.assign(d->max_timeouts, 0);
        for (uint32_t n = 0; n < d->n_nodes; ++n) hashes[n] = 0;
        if (o->live) gen = mk_stdgen(o->live->seed);
        res.status = TW_REP_RUNNING;
    }

    bool queue_empty() const { return mode == 0 ? cq.empty() : pq.empty(); }
    size_t queue_size() const { return mode == 0 ? cq.size() : pq.size(); }

    void hash(uint32_t node, uint32_t kind, int64_t val) {
        hashes[node] += tw_term(cur, kind, val);
        if (o->terms && o->terms_n < o->terms_cap) o->terms[o->terms_n] = two_term{cur, node, kind, val};
        if (o->terms) ++o->terms_n;
    }

    void fail(uint32_t status) {
        if (res.status == TW_REP_RUNNING) res.status = status;
    }

    // The engine's counters are 32-bit; reaching the top is a status, never a
    // silent wrap (the reference's counters are unbounded Integers).
    uint64_t next_seq() {
        // (TW_TIE_FORKFIRST keys spend bit 31 on the child mark: 31-bit counter)
        if (seq >= (cq.tie == TW_TIE_FORKFIRST ? 0x7FFFFFFFull : 0xFFFFFFFFull)) fail(TW_REP_ERR_COUNTER);
        else ++seq;
        return seq;
    }

    void enqueue(Thread* th, int64_t t, bool child = false) {
        Event e{t, next_seq() | (child && cq.tie == TW_TIE_FORKFIRST ? kChildMark : 0ull), th};
        if (mode == 0) cq.insert(e);
        else pq.insert(e);
    }

    Thread* new_thread(uint32_t pc, uint32_t node) {
        if (live_slots >= d->max_slots) {
            fail(TW_REP_ERR_SLOTS);
            return nullptr;
        }
        if (threads_counter >= 0xFFFFFFFFull) {
            fail(TW_REP_ERR_COUNTER);
            return nullptr;
        }
        ++live_slots;
        auto th = std::make_unique<Thread>();
        th->tid = threads_counter++;  // getNextThreadId, TimedT.hs:288-289
        th->pc = pc;
        th->node = node;
        Thread* p = th.get();
        by_tid.push_back(std::move(th));
        ++res.threads;
        return p;
    }

    void die(Thread* th) {
        th->alive = false;
        --live_slots;
        if (bind[th->node] && bind_owner[th->node] == th->tid) {
            bind[th->node] = 0;
            bind_owner[th->node] = UINT64_MAX;
        }
    }

    static int64_t ref_of(const Thread* th) { return (int64_t)(th->tid << 32); }

    // fork (TimedT.hs:326-342): child queued at now, parent `wait (for 1 mcs)`.
    Thread* fork(Thread* parent, uint32_t pc, uint32_t node, const int64_t regs[4]) {
        Thread* c = new_thread(pc, node);
        if (!c) return nullptr;
        for (int i = 0; i < 4; ++i) c->r[i] = regs[i];
        enqueue(c, cur, true);
        return c;
    }

    // throwTo (TimedT.hs:357-368)
    void throw_to(uint64_t tid, uint32_t code, int64_t val) {
        if (mode == 0) {
            Thread* t = tid < by_tid.size() ? by_tid[tid].get() : nullptr;  // dead => freed
            if (t && t->hpos >= 0) cq.restamp(t, cur, next_seq());
        } else {
            std::vector<Event> evs = pq.drain_ascending();  // PQ.toList
            for (Event& e : evs)
                if (e.th->tid == tid) e.t = cur;               // map modifyRequired
            pq.from_list(evs);                                 // PQ.fromList
        }
        if (async_exc.find(tid) == async_exc.end()) async_exc[tid] = Exc{code, val};  // old <|> new
    }

    // Raise `code` at the thread's current point; unwinding through finally
    // frames sets their done flag.  Returns true if a catch frame took it.
    bool unwind(Thread* th, uint32_t code, int64_t val) {
        while (th->nfr > 0) {
            Frame f = th->fr[--th->nfr];
            if (f.mask == 0) {
                if (f.pc < tmo_done.size()) tmo_done[f.pc] = 1;
                continue;
            }
            if (f.mask & (1u << code)) {
                th->pc = f.pc;
                th->r[0] = val;
                th->r[3] = code;
                return true;
            }
        }
        if (th->is_main) res.main_exc = code;  // caught by runTimedT's `try`
        die(th);                               // forked: threadKilledNotifier
        return false;
    }

    // BinaryP transmission time (tw_scenario_desc.msg_bytes / link_bw)
    int64_t tx_us(uint64_t link, uint32_t kind) const {
        if (!d->msg_bytes || !d->link_bw || kind >= d->n_msg_kinds) return 0;
        uint64_t bw = d->link_bw[link];
        if (!bw) return 0;
        return (int64_t)(((uint64_t)d->msg_bytes[kind] * 1000000ull + bw - 1) / bw);
    }

    uint32_t link_entry(uint32_t link) {
        uint32_t ord = link_ord[link]++;
        two_live_delays* lv = o->live;
        if (lv && lv->kind[link] != 0) {
            int64_t dly = lv->kind[link] == 1 ? lv->lo[link] : stdgen_range(gen, lv->lo[link], lv->hi[link]);
            uint32_t e = (uint32_t)dly & 0x7fffffffu;
            if (lv->record) {
                if (ord < lv->record_depth) lv->record[(size_t)link * lv->record_depth + ord] = e;
                else lv->record_overflow = 1;
            }
            return e;
        }
        if (!d->link_table) return 0;
        size_t idx = ((size_t)link * d->link_depth + ord % d->link_depth) * d->n_replicas + replica;
        return d->link_table[idx];
    }

    // Run a thread's continuation until it yields (wait/fork) or ends.
    void step(Thread* th) {
        th->started = true;
        const int64_t* K = d->consts;
        for (uint32_t n = 0; n < kStepCap; ++n) {
            if (th->pc >= d->n_insns) { fail(TW_REP_ERR_INSN); return; }
            tw_insn in = d->insns[th->pc];
            uint32_t op = in.w0 & 0xFF, a = (in.w0 >> 8) & 0xFF, b = in.w0 >> 16;
            int32_t imm = in.imm;
            int64_t* r = th->r;
            uint32_t ra = a & 3;
            ++th->pc;
            // fused `NSTORE a` after an ALU op (TW_ALU_NSTORE, timewarp.h)
            auto alu_nstore = [&] {
                if (b & TW_ALU_NSTORE) {
                    node_vars[(size_t)th->node * 4 + (b & 3)] = r[ra];
                    ++th->pc;
                }
            };
            switch (op) {
            case TW_OP_NOP: break;
            case TW_OP_END:
                die(th);
                return;
            case TW_OP_WAIT_REL:
                enqueue(th, cur + K[imm]);
                return;
            case TW_OP_WAIT_ABS:
                enqueue(th, std::max(cur, K[imm]));
                return;
            case TW_OP_WAIT_REG:
                enqueue(th, cur + std::max<int64_t>(r[ra], 0));
                return;
            case TW_OP_FORK: {
                uint32_t node = b == 0xFFFF ? th->node : (uint32_t)r[b & 3];
                if (node >= d->n_nodes) { fail(TW_REP_ERR_INSN); return; }
                Thread* c = fork(th, (uint32_t)imm, node, r);
                if (!c) return;
                r[ra] = ref_of(c);
                enqueue(th, cur + 1);
                return;
            }
            case TW_OP_MYTID: r[ra] = ref_of(th); break;
            case TW_OP_THROW_TO:
                throw_to((uint64_t)r[ra] >> 32, b & 0xFF, r[(b >> 8) & 3]);
                break;
            case TW_OP_THROW:
                if (!unwind(th, b & 0xFF, r[(b >> 8) & 3])) return;
                break;
            case TW_OP_CATCH:
                if ((uint32_t)th->nfr >= max_frames) { fail(TW_REP_ERR_FRAMES); return; }
                th->fr[th->nfr++] = Frame{(uint16_t)b, (uint16_t)imm};
                break;
            case TW_OP_UNCATCH:
                if (th->nfr == 0 || th->fr[th->nfr - 1].mask == 0) { fail(TW_REP_ERR_INSN); return; }
                --th->nfr;
                break;
            case TW_OP_SETI: r[ra] = imm; alu_nstore(); break;
            case TW_OP_SETK: r[ra] = K[imm]; alu_nstore(); break;
            case TW_OP_ADDI: r[ra] += imm; alu_nstore(); break;
            case TW_OP_MULI: r[ra] *= imm; alu_nstore(); break;
            case TW_OP_MOV: r[ra] = r[b & 3]; break;
            case TW_OP_ADD: r[ra] += r[b & 3]; break;
            case TW_OP_SUB: r[ra] -= r[b & 3]; break;
            case TW_OP_MODI: {
                int64_t m = r[ra] % imm;
                r[ra] = m < 0 ? m + imm : m;
                break;
            }
            case TW_OP_JMP: th->pc = (uint32_t)imm; break;
            case TW_OP_JEQ: if (r[ra] == r[b & 3]) th->pc = (uint32_t)imm; break;
            case TW_OP_JNE: if (r[ra] != r[b & 3]) th->pc = (uint32_t)imm; break;
            case TW_OP_JLT: if (r[ra] < r[b & 3]) th->pc = (uint32_t)imm; break;
            case TW_OP_JLE: if (r[ra] <= r[b & 3]) th->pc = (uint32_t)imm; break;
            case TW_OP_JEQI: if (r[ra] == (int16_t)b) th->pc = (uint32_t)imm; break;
            case TW_OP_JNEI: if (r[ra] != (int16_t)b) th->pc = (uint32_t)imm; break;
            case TW_OP_NOW: r[ra] = cur; alu_nstore(); break;
            case TW_OP_NODE: r[ra] = th->node; alu_nstore(); break;
            case TW_OP_NLOAD: r[ra] = node_vars[(size_t)th->node * 4 + (b & 3)]; break;
            case TW_OP_NSTORE: node_vars[(size_t)th->node * 4 + (b & 3)] = r[ra]; break;
            case TW_OP_NLOADX:
            case TW_OP_NSTOREX: {
                uint64_t node = (uint64_t)r[(b >> 8) & 3];
                if (node >= d->n_nodes) { fail(TW_REP_ERR_INSN); return; }
                int64_t& v = node_vars[node * 4 + (b & 3)];
                if (op == TW_OP_NLOADX) r[ra] = v;
                else v = r[ra];
                break;
            }
            case TW_OP_LINK: r[ra] = (int64_t)d->out_off[th->node] + imm; break;
            case TW_OP_RLINK: {
                uint64_t l = (uint64_t)r[b & 3];
                if (l >= d->n_links) { fail(TW_REP_ERR_INSN); return; }
                r[ra] = (int64_t)d->link_rev[l];
                break;
            }
            case TW_OP_SEND: {
                // fused LINK / RLINK (timewarp.h TW_SEND_VIA_*): the pair's first
                // instruction, then this send, then past the pair's SEND
                if (b & TW_SEND_VIA_LINK) {
                    r[ra] = (int64_t)d->out_off[th->node] + imm;
                    ++th->pc;
                } else if (b & TW_SEND_VIA_RLINK) {
                    uint64_t l = (uint64_t)r[(b >> 12) & 3];
                    if (l >= d->n_links) { fail(TW_REP_ERR_INSN); return; }
                    r[ra] = (int64_t)d->link_rev[l];
                    ++th->pc;
                }
                uint64_t link = (uint64_t)r[ra];
                if (link >= d->n_links) { fail(TW_REP_ERR_INSN); return; }
                uint32_t kind = b & 0xFF;
                int64_t payload = r[(b >> 8) & 3];
                uint32_t e = link_entry((uint32_t)link);
                if (e & TW_LINK_DROP) {  // nastiness: message lost, no thread, no yield
                    ++res.dropped;
                    hash(th->node, TW_KIND_DROP | kind, payload);
                    break;
                }
                // delay = link-table delay + BinaryP transmission time of the message
                int64_t regs[4] = {payload, (int64_t)link, (int64_t)(e & 0x7fffffffu) + tx_us(link, kind),
                                   (int64_t)kind};
                // schedule (after d) (deliver ..) = fork_ (wait (after d) >> deliver ..)
                if (!fork(th, TW_PC_DELIVER_STUB, th->node, regs)) return;
                enqueue(th, cur + 1);
                return;
            }
            case TW_OP_DELIVER: {
                uint64_t link = (uint64_t)r[1];
                uint32_t kind = (uint32_t)r[3];
                uint32_t dst = d->link_dst[link];
                uint32_t set = bind[dst];
                uint32_t lpc = TW_PC_NONE;
                if (set && kind < d->n_msg_kinds) lpc = d->listener_pc[(size_t)(set - 1) * d->n_msg_kinds + kind];
                if (lpc == TW_PC_NONE) {
                    ++res.undeliverable;
                    hash(dst, TW_KIND_UNDELIV | kind, r[0]);
                    break;
                }
                ++res.delivered;
                hash(dst, TW_KIND_RECV | kind, r[0]);
                int64_t regs[4] = {r[0], (int64_t)link, (int64_t)th->node, (int64_t)kind};
                if (lpc & TW_LPC_INLINE) {
                    // ForkStrategy `const id` (MonadDialog.hs:114-117): the handler runs
                    // in this thread, on the destination node, with the handler's registers
                    for (int i = 0; i < 4; ++i) r[i] = regs[i];
                    th->node = dst;
                    th->pc = lpc & ~TW_LPC_INLINE;
                    break;
                }
                // ForkStrategy default fork_ (MonadDialog.hs:317)
                if (!fork(th, lpc, dst, regs)) return;
                enqueue(th, cur + 1);
                return;
            }
            case TW_OP_LISTEN:
                if ((uint32_t)imm >= d->n_listener_sets) { fail(TW_REP_ERR_INSN); return; }
                bind[th->node] = (uint32_t)imm + 1;
                bind_owner[th->node] = b ? th->tid : UINT64_MAX;
                break;
            case TW_OP_UNLISTEN:
                bind[th->node] = 0;
                bind_owner[th->node] = UINT64_MAX;
                break;
            case TW_OP_TRACE:
                hash(th->node, TW_KIND_TRACE | ((uint32_t)imm & 0xFFFF), r[ra]);
                if (o->traces && o->traces_n < o->traces_cap)
                    o->traces[o->traces_n] = two_term{cur, th->node, (uint32_t)imm, r[ra]};
                if (o->traces) ++o->traces_n;
                if (b & TW_TRACE_PAIR) {  // fused second TRACE (timewarp.h)
                    const uint32_t t2 = b & 0x1FFF, a2 = (b >> 13) & 3;
                    hash(th->node, TW_KIND_TRACE | t2, r[a2]);
                    if (o->traces && o->traces_n < o->traces_cap)
                        o->traces[o->traces_n] = two_term{cur, th->node, t2, r[a2]};
                    if (o->traces) ++o->traces_n;
                    ++th->pc;
                }
                break;
            case TW_OP_TMO_BEGIN: {
                if (tmo_ctr >= d->max_timeouts) { fail(TW_REP_ERR_INSN); return; }
                uint32_t e = tmo_ctr++;
                tmo_done[e] = 0;
                r[ra] = e;
                int64_t regs[4] = {ref_of(th), (int64_t)e, K[imm], 0};
                if (!fork(th, TW_PC_WATCHDOG_STUB, th->node, regs)) return;
                enqueue(th, cur + 1);
                return;
            }
            case TW_OP_TMO_PUSH:
                if ((uint32_t)th->nfr >= max_frames) { fail(TW_REP_ERR_FRAMES); return; }
                th->fr[th->nfr++] = Frame{0, (uint16_t)r[ra]};
                break;
            case TW_OP_TMO_END: {
                if (th->nfr == 0 || th->fr[th->nfr - 1].mask != 0) { fail(TW_REP_ERR_INSN); return; }
                Frame f = th->fr[--th->nfr];
                tmo_done[f.pc] = 1;
                break;
            }
            case TW_OP_TMO_FIRE:
                if (!tmo_done[(size_t)r[1]]) throw_to((uint64_t)r[0] >> 32, TW_EXC_TIMEOUT, 0);
                break;
            default:
                fail(TW_REP_ERR_INSN);
                return;
            }
            if (res.status != TW_REP_RUNNING) return;
        }
        fail(TW_REP_ERR_INSN);
    }

    void reap(Thread* th) {
        if (!th->alive) by_tid[th->tid].reset();  // a dead thread has no queued event
    }

    void run_main() {
        Thread* m = new_thread(d->main_pc, d->main_node);
        m->is_main = true;
        if (d->main_regs)
            for (int i = 0; i < 4; ++i) m->r[i] = d->main_regs[(size_t)replica * 4 + i];
        step(m);  // runInSandbox main (TimedT.hs:237): no pop
        reap(m);
    }

    void loop() {
        while (res.status == TW_REP_RUNNING && !queue_empty()) {  // whileM_ notDone
            if (o->max_events && res.events >= o->max_events) return;
            Event ev;
            if (mode == 0) {
                // peek for t_end without popping
                ev = cq.pop();
                if (ev.t > o->t_end) { cq.insert(ev); return; }
            } else {
                if (pq.top().t > o->t_end) return;
                ev = pq.pop();                                 // PQ.minView
            }
            cur = ev.t;                                        // curTime .= timestamp
            ++res.events;
            res.final_t = cur;
            Thread* th = ev.th;
            auto it = async_exc.find(th->tid);                 // asyncExceptions . at tid <<.= Nothing
            bool has_exc = it != async_exc.end();
            Exc ex{};
            if (has_exc) {
                ex = it->second;
                async_exc.erase(it);
            }
            if (has_exc) {
                hash(th->node, TW_KIND_EXC | ex.code, 0);
                if (!th->started && !th->is_main) {
                    // thrown before the forked action (and its catch) begins:
                    // ctx handlers = [] => escapes launchTimedT (TimedT.hs:252-263)
                    res.status = TW_REP_ABORTED;
                    res.main_exc = ex.code;
                    return;
                }
                if (unwind(th, ex.code, ex.val)) step(th);
            } else {
                hash(th->node, TW_KIND_RESUME | th->pc, 0);
                step(th);
            }
            reap(th);
        }
        if (res.status == TW_REP_RUNNING && queue_empty()) res.status = TW_REP_DONE;
    }
};

}  // namespace

extern "C" {

int two_run(const tw_scenario_desc* d, uint32_t replica, two_opts* o, tw_replica_result* res,
            uint64_t* hashes) {
    if (!d || !o || !res || !hashes || replica >= d->n_replicas) return TW_ERR_INVALID;
    o->terms_n = 0;
    o->traces_n = 0;
    Sim s(d, replica, o, hashes);
    s.run_main();
    s.loop();
    *res = s.res;
    return TW_OK;
}

// Replicas [r0, r1) on `nthreads` host threads (one replica per worker at a
// time), canonical or pqueue mode, no logs.  The CPU baseline.
int two_run_batch(const tw_scenario_desc* d, uint32_t r0, uint32_t r1, int mode, int nthreads,
                  tw_replica_result* res, uint64_t* hashes) {
    if (!d || r1 > d->n_replicas || r0 > r1) return TW_ERR_INVALID;
    if (nthreads < 1) nthreads = 1;
    std::vector<std::thread> pool;
    std::atomic<uint32_t> next{r0};
    for (int w = 0; w < nthreads; ++w) {
        pool.emplace_back([&]() {
            for (;;) {
                uint32_t r = next.fetch_add(1);
                if (r >= r1) return;
                two_opts o{};
                o.mode = mode;
                o.t_end = INT64_MAX;
                Sim s(d, r, &o, hashes + (size_t)(r - r0) * d->n_nodes);
                s.run_main();
                s.loop();
                res[r - r0] = s.res;
            }
        });
    }
    for (auto& t : pool) t.join();
    return TW_OK;
}

// random-1.1 StdGen helpers, exported for the golden-vector tests.
void two_stdgen_draws(int64_t seed, int64_t lo, int64_t hi, int64_t* out, size_t n) {
    StdGen g = mk_stdgen(seed);
    for (size_t i = 0; i < n; ++i) out[i] = stdgen_range(g, lo, hi);
}
void two_stdgen_next(int64_t seed, int32_t* out, size_t n, int32_t* s1s2) {
    StdGen g = mk_stdgen(seed);
    if (s1s2) { s1s2[0] = g.s1; s1s2[1] = g.s2; }
    for (size_t i = 0; i < n; ++i) out[i] = stdgen_next(g);
}

// pqueue transcription self-test hook: ops[i] >= 0 inserts key ops[i] with
// payload id i, ops[i] == -1 pops (minView) and records the payload id.
// Returns the number of ids written.
size_t two_pqueue_order(const int64_t* ops, size_t n, int64_t* out_ids) {
    struct KV { int64_t k; int64_t id; };
    struct LE { bool operator()(const KV& a, const KV& b) const { return a.k <= b.k; } };
    PQueueMin<KV, LE> q;
    size_t m = 0;
    for (size_t i = 0; i < n; ++i) {
        if (ops[i] >= 0) q.insert(KV{ops[i], (int64_t)i});
        else if (!q.empty()) out_ids[m++] = q.pop().id;
    }
    return m;
}

}  // extern "C"
