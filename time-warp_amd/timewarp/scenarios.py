"""Scenario builders for the BASELINE.json configs, lowered to thread programs.

Each builder restates a reference scenario as per-node handler state machines
(see program.py for the API mapping) and draws its link tables from random-1.1
StdGen, one generator per replica, so every trace is deterministic: on the
host (stdgen.py) or, with ``drawer=engine.draw_link_table``, the same draw on
the GPU (tw_draw_link_table).

  token_ring  — examples/token-ring/Main.hs (configs 1 and 3)
  ping_pong   — examples/ping-pong/Main.hs re-hosted on emulation (config 2)
  hotspot     — bench/Network Sender/Receiver request/response (config 5)
"""
from __future__ import annotations

import numpy as np

from . import isa
from .program import Program
from .scenario import Scenario, Topology
from .stdgen import StdGenVec
from .timeunits import after, at, for_, ms, sec

# trace tags (logInfo / logError / logMeasure points of the reference scenarios)
TAG_CREATE_TOKEN = 1     # token-ring/Main.hs:134  "Creating token"
TAG_GOT_TOKEN = 2        # token-ring/Main.hs:138  "Got token with value"
TAG_NOTE = 3             # token-ring/Main.hs:200-204 noteTokenMethod
TAG_WRONG_VALUE = 4      # token-ring/Main.hs:206-208 "Wrong token value"
TAG_NO_PROGRESS = 5      # token-ring/Main.hs:184-187 "Token value hasn't changed"
TAG_PING = 6             # ping-pong/Main.hs:73-75  "Get Ping"; bench PingReceived
TAG_PONG = 7             # ping-pong/Main.hs:64-66  "Get Pong"; bench PongReceived
TAG_PING_SENT = 8        # bench/Network/Sender/Main.hs:60 logMeasure PingSent
TAG_PONG_SENT = 9        # bench/Network/Receiver/Main.hs:36 logMeasure PongSent

EXC_VALUE_RECEIVED = isa.EXC_USER0  # data SignalException = ValueReceived Int (token-ring/Main.hs:156)


def _capped(n: int) -> int:
    return int(min(n, 0xFFFFFFFF))


# -------------------------------------------------------------- link tables
def draw_table(n_links: int, n_replicas: int, drawn_links, lo, hi, link_depth: int = 1, drop_log2: int = 0,
               seed_base: int = 0, drawer=None) -> np.ndarray:
    """The scenarios' link-table draw (examples/token-ring/Main.hs:60,77:
    ``mkStdGen`` + ``getRandomTR``), one StdGen per replica (seed_base + r):
    for each link of ``drawn_links`` in ascending order, ``link_depth``
    entries, each a randomR(lo, hi) delay followed by a drop coin when
    drop_log2 > 0 (dropped when 0).  Other links hold ``lo``.  ``drawer`` =
    ``engine.draw_link_table`` runs the same draw on the GPU
    (tw_draw_link_table); the default is the host draw of stdgen.py."""
    drawn = np.zeros(n_links, np.uint8)
    drawn[np.asarray(drawn_links, dtype=np.int64)] = 1
    lo = np.broadcast_to(np.asarray(lo, dtype=np.int64), (n_links,)).copy()
    hi = np.broadcast_to(np.asarray(hi, dtype=np.int64), (n_links,)).copy()
    if drawer is not None:
        return drawer(n_replicas, drawn, lo, hi, link_depth=link_depth, drop_log2=drop_log2, seed_base=seed_base)
    table = np.empty((n_links, link_depth, n_replicas), np.uint32)
    table[:] = lo.astype(np.uint32)[:, None, None]
    g = StdGenVec(seed_base + np.arange(n_replicas, dtype=np.int64))
    for l in np.nonzero(drawn)[0].tolist():
        for k in range(link_depth):
            dly = g.range(int(lo[l]), int(hi[l])).astype(np.uint32)
            if drop_log2:
                u = g.range(0, (1 << drop_log2) - 1)
                dly = np.where(u == 0, dly | np.uint32(isa.LINK_DROP), dly)
            table[l, k, :] = dly
    return table


# --------------------------------------------------------------- token ring
def token_ring(n_nodes: int = 16, n_replicas: int = 1, launch_duration: int = sec(20),
               token_passing_delay: int = sec(3), allowed_progress_delay: int = sec(5),
               network_delay=(ms(1), ms(5)), drop_log2: int = 0, seed_base: int = 0,
               link_depth: int = 1, near_horizon_us: int = sec(10), drawer=None) -> Scenario:
    """examples/token-ring/Main.hs lowered.

    Node ids: ring nodes 0..N-1 are the reference's ``no = 1..N``
    (nodePort = 2000+no, :87-88), node N is the observer (port 5000, :163-164),
    node N+1 hosts the main thread.  Out-links: ring node i -> [(i+1) mod N,
    observer].  ``call`` (MonadRpc, absent) is lowered to a one-way send.
    Delays (:73-77): observer links ConnectedIn 0; ring links U[1 ms, 5 ms];
    optional drop with probability 2^-drop_log2 per send (config 3 nastiness).
    """
    N = int(n_nodes)
    OBS, SYS = N, N + 1
    p = Program()
    K_TOKEN, K_NOTE = p.kind("token"), p.kind("noteToken")
    ring_set = p.listener_set({"token": "accept_token"})
    obs_set = p.listener_set({"noteToken": "note_token"})

    # scenario (main thread), :63-72
    c = p.function("main")
    c.seti(0, 0).seti(2, N)
    loop = c.here()
    c.fork("launch_node", ref=1, node_reg=0)          # fork $ launchNode no
    c.addi(0, 1).jlt(0, 2, loop)
    c.seti(0, OBS)
    c.fork_("launch_observer", node_reg=0)            # fork_ launchObserver
    c.end()

    # launchNode no, :104-135
    c = p.function("launch_node")
    c.fork("worker", ref=1)                           # wtid <- fork worker
    c.nstore(1, 0)                                    # (acceptToken closes over wtid)
    c.fork("server", ref=2)                           # stid <- fork server
    c.schedule(at(launch_duration), "kill_pair")      # schedule (at launchDuration) kill
    c.node(0)
    done = c.label()
    c.jnei(0, 0, done)                                # when (no == 1)
    c.invoke(after(sec(1)))                           # invoke (after 1 sec)
    c.trace(TAG_CREATE_TOKEN, 0)
    c.seti(0, 1)
    c.link(1, 0).send(1, K_TOKEN, 0)                  # initPassingToken 1
    c.bind(done)
    c.end()

    c = p.function("kill_pair")                       # mapM_ killThread [r1, r2]
    c.kill_thread(1).kill_thread(2).end()

    # worker: forever $ catch sleepForever onValueReceived, :110-112, 137-147
    c = p.function("worker")
    c.catch_(1 << EXC_VALUE_RECEIVED, "on_value")
    c.sleep_forever()
    c = p.function("on_value")                        # r0 = v
    c.trace(TAG_GOT_TOKEN, 0)
    c.link(1, 1).send(1, K_NOTE, 0)                   # execClient observer (noteTokenCall v)
    c.wait(for_(token_passing_delay))                 # wait (for tokenPassingDelay)
    c.addi(0, 1)
    c.link(1, 0).send(1, K_TOKEN, 0)                  # initPassingToken (v + 1)
    c.jmp("worker")

    # server: serve (no ^. nodePort) [method "token" (acceptToken wtid)], :116-122
    c = p.function("server")
    c.listen(ring_set, owned=True)
    c.sleep_forever()
    c = p.function("accept_token")                    # acceptToken tid value, :152-154
    c.nload(2, 0).throw_to(2, EXC_VALUE_RECEIVED, 0).end()

    # launchObserver, :166-194
    c = p.function("launch_observer")
    c.fork("obs_server", ref=1)
    c.fork("checker", ref=2)
    c.schedule(at(launch_duration), "kill_pair")
    c.end()
    c = p.function("obs_server")
    c.listen(obs_set, owned=True)
    c.sleep_forever()
    c = p.function("checker")                         # forever $ wait 1 sec; check progress
    chk = c.here()
    c.wait(for_(sec(1)))
    c.nload(0, 0).now(1).sub(1, 0).seti(2, allowed_progress_delay)
    c.jle(1, 2, chk)
    c.nload(3, 1).trace(TAG_NO_PROGRESS, 3)
    c.jmp(chk)
    c = p.function("note_token")                      # noteTokenMethod, :197-208
    c.now(1).nload(2, 1).nstore(1, 0).nstore(0, 1)
    c.trace(TAG_NOTE, 0)
    ok = c.label()
    c.addi(2, 1).jeq(0, 2, ok)
    c.trace(TAG_WRONG_VALUE, 0)
    c.bind(ok)
    c.end()

    img = p.finalize()
    out = [[(i + 1) % N, OBS] for i in range(N)] + [[], []]
    topo = Topology.from_out_lists(N + 2, out)
    L = topo.n_links

    # Delays: ring links (even ids) random, observer links (odd ids) 0
    ring_links = np.arange(0, 2 * N, 2)
    lo = np.zeros(L, np.int64)
    hi = np.zeros(L, np.int64)
    lo[ring_links], hi[ring_links] = network_delay
    live_kind = np.zeros(L, np.uint32)
    live_kind[ring_links] = 2
    live_kind[ring_links + 1] = 1
    live_lo, live_hi = lo.copy(), hi.copy()
    table = draw_table(L, n_replicas, ring_links, lo, hi, link_depth=link_depth, drop_log2=drop_log2,
                       seed_base=seed_base, drawer=drawer)

    hops = launch_duration // max(1, token_passing_delay) + 2
    max_slots = 3 * N + 64
    return Scenario(
        name=f"token_ring_n{N}",
        image=img, topo=topo, n_replicas=n_replicas,
        main_pc=img.pc_of("main"), main_node=SYS,
        link_table=table, max_slots=_capped(max_slots),
        queue_capacity=_capped(max_slots + 2 * N + 4 * hops + 256),
        run_capacity=_capped(2 * N + 4 * hops + 256),
        near_horizon_us=near_horizon_us,
        meta=dict(config="token_ring", n_nodes=N, launch_duration=launch_duration,
                  drop_log2=drop_log2, seed_base=seed_base,
                  # batched node-partitioned mode (Engine.load_lpb): a ring node holds
                  # launchNode's threads (worker, server, killer, the token's
                  # deliverer and handler), the observer its server, checker, killer
                  # and note deliveries; main's spawn pairs are a tick's records.
                  # The observer's 0 µs links make it a phase-1 node.  At most
                  # six threads and their events per node: 8 slots and 8 far
                  # entries behind the 8 on-chip ones (~1.7 KB per lane, so
                  # 32,768 replicas x 4,098 nodes fit one GPU's HBM)
                  lp_inbox_cap=np.array([4] * N + [8, 1], np.uint32),
                  lp_max_slots=8, lp_queue_capacity=8,
                  lp_outbox_cap=min(1 << 27, (2 * (N + 2) + 64) * n_replicas)),
        live_kind=live_kind, live_lo=live_lo, live_hi=live_hi,
    )


# ---------------------------------------------------------------- ping-pong
def ping_pong(n_replicas: int = 1, round_trips: int = 1, network_delay=(ms(1), ms(5)),
              seed_base: int = 0, near_horizon_us: int = sec(10), drawer=None) -> Scenario:
    """examples/ping-pong/Main.hs re-hosted on the emulated transfer.

    Node 0 = "ping" (listens AtPort 4444), node 1 = "pong" (AtPort 5555),
    node 2 hosts main.  ping: wait 2 s, send Ping, listen for Pong (:57-67);
    pong: listen for Ping, reply Pong (:69-77).  ``round_trips`` > 1 re-sends
    Ping on each Pong (throughput extension; 1 reproduces the example).
    Per-replica per-link constant delays ~ U[1 ms, 5 ms] from mkStdGen(replica),
    drawn ping->pong then pong->ping.
    """
    p = Program()
    K_PING, K_PONG = p.kind("Ping"), p.kind("Pong")
    ping_set = p.listener_set({"Pong": "on_pong"})
    pong_set = p.listener_set({"Ping": "on_ping"})

    c = p.function("main")
    c.seti(0, 0).fork_("ping_main", node_reg=0)
    c.seti(0, 1).fork_("pong_main", node_reg=0)
    c.end()

    c = p.function("ping_main")
    c.wait(for_(sec(2)))                              # wait (for 2 sec)
    c.seti(0, 0).link(1, 0).send(1, K_PING, 0)        # send (localhost, 5555) Ping
    c.listen(ping_set)                                # listen (AtPort 4444) [...]
    c.end()

    c = p.function("pong_main")
    c.listen(pong_set)                                # listen (AtPort 5555) [...]
    c.end()

    c = p.function("on_ping")                         # \Ping -> log; send (localhost,4444) Pong
    c.trace(TAG_PING, 0)
    c.link(2, 0).send(2, K_PONG, 0)
    c.end()

    c = p.function("on_pong")                         # \Pong -> log
    c.trace(TAG_PONG, 0)
    c.addi(0, 1).seti(2, round_trips)
    fin = c.label()
    c.jle(2, 0, fin)
    c.link(1, 0).send(1, K_PING, 0)
    c.bind(fin)
    c.end()

    img = p.finalize()
    topo = Topology.from_out_lists(3, [[1], [0], []])
    table = draw_table(2, n_replicas, [0, 1], *network_delay, seed_base=seed_base, drawer=drawer)
    return Scenario(
        name="ping_pong", image=img, topo=topo, n_replicas=n_replicas,
        main_pc=img.pc_of("main"), main_node=2, link_table=table,
        max_slots=16, queue_capacity=64, near_horizon_us=near_horizon_us,
        meta=dict(config="ping_pong", round_trips=round_trips, seed_base=seed_base),
    )


# ------------------------------------------------------------------ hotspot
def hotspot(n_senders: int = 256, n_replicas: int = 1, msg_num: int = 1000, msg_rate: int = 1000,
            duration_s: int = 10, network_delay=(ms(1), ms(5)), seed_base: int = 0,
            near_horizon_us: int = sec(10), fork_strategy: str = "fork", payload_bytes: int = 0,
            bandwidth_bytes_per_s: float = 0.0, probe_traces: int = 0, probe_loads: int = 0,
            drop_log2: int = 0, receiver_counter: bool = False, drawer=None) -> Scenario:
    """bench/Network many-senders -> one-receiver request/response.

    Sender (Sender/Main.hs:34-64): listen for Pong, then per message
    ``wait (for sendDelay)`` with sendDelay = 10^6 / msgRate µs (:38-39),
    stop once the work timer exceeds ``duration`` (:52-53), send Ping msgId;
    finally ``wait (for 1 sec)`` and close.  Receiver (Receiver/Main.hs:32-41):
    listen, on Ping reply Pong, stop after ``duration``.  Node i < S = sender i,
    node S = receiver, node S+1 hosts main.  Links: i -> S (id i), S -> i (id S+i).

    ``fork_strategy="inline"`` dispatches Ping and Pong in place in the
    delivering thread (ForkStrategy `const id`, MonadDialog.hs:114-117) instead
    of the default `fork_` (MonadDialog.hs:317): two pops fewer per delivery.

    ``probe_traces`` / ``probe_loads`` (diagnostics only, tools/pass_probe.py)
    add that many trace / node-variable load instructions to the Ping handler:
    the receiver's cost per instruction pass and per dependent memory load.

    ``drop_log2 > 0`` drops each send with probability 2^-drop_log2 (tests);
    ``receiver_counter`` makes the Ping handler count its pings in a node
    variable (a stateful handler: tests of the batched delivery's classifier).

    ``bandwidth_bytes_per_s > 0`` adds each message's transmission time to its
    link delay: the BinaryP wire size of `Ping/Pong MsgId Payload` with a
    ``payload_bytes`` payload (timewarp.wire, Message.hs:155-202,
    Commons.hs:49-70).
    """
    if fork_strategy not in ("fork", "inline"):
        raise ValueError(f"fork_strategy must be 'fork' or 'inline', not {fork_strategy!r}")
    inl = fork_strategy == "inline"
    S = int(n_senders)
    RECV, SYS = S, S + 1
    send_delay = 1_000_000 // msg_rate
    p = Program()
    K_PING, K_PONG = p.kind("Ping"), p.kind("Pong")
    recv_set = p.listener_set({"Ping": "on_ping"}, inline=("Ping",) if inl else ())
    send_set = p.listener_set({"Pong": "on_pong"}, inline=("Pong",) if inl else ())

    c = p.function("main")
    c.seti(0, RECV).fork_("receiver_main", node_reg=0)
    c.seti(0, 0).seti(2, S)
    loop = c.here()
    c.fork("sender_main", ref=1, node_reg=0)
    c.addi(0, 1).jlt(0, 2, loop)
    c.end()

    c = p.function("receiver_main")
    c.listen(recv_set)                                # stopper <- listen (AtPort port) [...]
    c.wait(for_(sec(duration_s)))                     # wait (for duration sec)
    c.unlisten()                                      # stopper
    c.end()

    c = p.function("on_ping")                         # Ping -> logMeasure; reply Pong
    for _ in range(int(probe_traces)):
        c.trace(TAG_PING, 0)
    for _ in range(int(probe_loads)):
        c.nload(3, 2)
    if receiver_counter:
        c.nload(3, 0).addi(3, 1).nstore(3, 0)
    c.trace(TAG_PING, 0)                              # logMeasure PingReceived mid
    c.trace(TAG_PONG_SENT, 0)                         # logMeasure PongSent mid
    c.reply_link(2, 1).send(2, K_PONG, 0)
    c.end()

    c = p.function("sender_main")
    c.listen(send_set)                                # listen (AtConnTo addr) [Pong -> ...]
    c.now(1).nstore(1, 0)                             # workTimer <- startTimer
    c.node(0).addi(0, 1)                              # msgIds [tid, tid+threadNum .. msgNum] (:40)
    top = c.here()
    stop = c.label()
    c.wait(for_(send_delay))                          # wait (for sendDelay)
    c.now(1).nload(3, 0).sub(1, 3).seti(3, sec(duration_s))
    c.jlt(3, 1, stop)                                 # when (working > duration) mzero
    c.trace(TAG_PING_SENT, 0)
    c.link(1, 0).send(1, K_PING, 0)                   # send addr (Ping sMsgId payload)
    c.addi(0, S).seti(2, S * msg_num)
    c.jle(0, 2, top)
    c.bind(stop)
    c.wait(for_(sec(1)))                              # wait (for 1 sec)  -- responses
    c.unlisten()                                      # sequence_ closeConns
    c.end()

    c = p.function("on_pong")
    c.trace(TAG_PONG, 0)
    c.end()

    img = p.finalize()
    out = [[RECV] for _ in range(S)] + [list(range(S)), []]
    topo = Topology.from_out_lists(S + 2, out)
    table = draw_table(topo.n_links, n_replicas, np.arange(topo.n_links), *network_delay, seed_base=seed_base,
                       drop_log2=drop_log2, drawer=drawer)
    if bandwidth_bytes_per_s > 0:
        from .wire import bench_message_size, transmission_us
        table[:S] += transmission_us(bench_message_size("Ping", payload_bytes), bandwidth_bytes_per_s)
        table[S:2 * S] += transmission_us(bench_message_size("Pong", payload_bytes), bandwidth_bytes_per_s)
    max_delay = int(table.max()) if table.size else int(network_delay[1])
    in_flight = (max_delay // max(1, send_delay) + 2) * 2
    max_slots = S * (in_flight + 2) + 64
    return Scenario(
        name=f"hotspot_s{S}" + ("_inline" if inl else ""), image=img, topo=topo, n_replicas=n_replicas,
        main_pc=img.pc_of("main"), main_node=SYS, link_table=table,
        max_slots=_capped(max_slots), queue_capacity=_capped(2 * max_slots + 256),
        run_capacity=_capped(2 * S + 64), near_horizon_us=near_horizon_us,
        meta=dict(config="hotspot", n_senders=S, msg_num=msg_num, msg_rate=msg_rate, payload_bytes=payload_bytes,
                  # batched node-partitioned mode (Engine.load_lpb): per-lane capacities;
                  # the receiver holds every ping in flight (<= max_delay / sendDelay + 2
                  # per sender), a sender its pongs, and a tick's records per replica are
                  # <= a ping and a pong per sender and window plus main's spawn pairs
                  lp_inbox_cap=np.array([32] * S + [min(2048, S * (max_delay // max(1, send_delay) + 2) + 64), 4],
                                        np.uint32),
                  lp_max_slots=64, lp_queue_capacity=128,
                  lp_outbox_cap=min(1 << 27, (8 * S + 2 * (S + 1) + 64) * n_replicas)),
    )


# --------------------------------------------------------------- gatekeeper
TAG_RAW = 10             # raw listener saw a message (MonadDialog.hs:226-256)
TAG_REQ = 11
TAG_ACK = 12


def gatekeeper(n_clients: int = 4, n_replicas: int = 1, msg_num: int = 20, junk_every: int = 4,
               network_delay=(ms(1), ms(5)), seed_base: int = 0, raw: bool = True,
               near_horizon_us: int = sec(10), drawer=None) -> Scenario:
    """A ``listenR`` server (MonadDialog.hs:226-256): the raw listener logs
    every message that reaches the port and returns True only for even
    payloads; the typed listener for `Req` then replies `Ack`.  Clients also
    send `Junk`, a name the server has no typed listener for: the reference
    still runs the raw listener for it (:240-244).

    Node i < C = client i, node C = server, node C+1 hosts main.  Client i
    sends Req with payload i*msg_num + m every 1 ms (m = 0..msg_num-1) and a
    Junk after every Req whose payload is -1 mod `junk_every`, then waits 1 s
    for Acks.  Links:
    i -> C (id i), C -> i (id C+i), per-link delays ~ U[1, 5] ms from
    mkStdGen(replica).  ``raw=False`` binds the same typed listener with a
    plain ``listen`` (every Req is answered; Junk ends in a handler thread
    that only logs "No listener", MonadDialog.hs:240-244)."""
    C = int(n_clients)
    SRV, SYS = C, C + 1
    p = Program()
    K_REQ, K_ACK, K_JUNK = p.kind("Req"), p.kind("Ack"), p.kind("Junk")

    def raw_listener(c, accept):
        c.trace(TAG_RAW, 0)                           # raw (header, raw) -> log it
        c.mov(2, 0).modi(2, 2)
        c.jeqi(2, 0, accept)                          # return (even payload)

    srv_set = p.listener_set({"Req": "on_req"}, raw=raw_listener if raw else None)
    cli_set = p.listener_set({"Ack": "on_ack"})

    c = p.function("main")
    c.seti(0, SRV).fork_("server_main", node_reg=0)
    c.seti(0, 0).seti(2, C)
    loop = c.here()
    c.fork_("client_main", node_reg=0)
    c.addi(0, 1).jlt(0, 2, loop)
    c.end()

    c = p.function("server_main")
    c.listen(srv_set)                                 # listenR (AtPort p) [Req] raw
    c.wait(for_(sec(10)))
    c.unlisten()
    c.end()

    c = p.function("on_req")
    c.trace(TAG_REQ, 0)
    c.reply_link(2, 1).send(2, K_ACK, 0)
    c.end()

    c = p.function("client_main")
    c.listen(cli_set)
    c.node(0).muli(0, msg_num)                        # r0 = first payload
    c.mov(1, 0).addi(1, msg_num)                      # r1 = end
    top = c.here()
    skip = c.label()
    c.wait(for_(ms(1)))
    c.link(2, 0).send(2, K_REQ, 0)
    c.mov(3, 0).modi(3, junk_every).jnei(3, junk_every - 1, skip)
    c.send(2, K_JUNK, 0)
    c.bind(skip)
    c.addi(0, 1).jlt(0, 1, top)
    c.wait(for_(sec(1)))
    c.unlisten()
    c.end()

    c = p.function("on_ack")
    c.trace(TAG_ACK, 0)
    c.end()

    img = p.finalize()
    out = [[SRV] for _ in range(C)] + [list(range(C)), []]
    topo = Topology.from_out_lists(C + 2, out)
    table = draw_table(topo.n_links, n_replicas, np.arange(topo.n_links), *network_delay, seed_base=seed_base,
                       drawer=drawer)
    max_slots = C * 24 + 64
    return Scenario(
        name=f"gatekeeper_c{C}" + ("" if raw else "_plain"), image=img, topo=topo, n_replicas=n_replicas,
        main_pc=img.pc_of("main"), main_node=SYS, link_table=table,
        max_slots=_capped(max_slots), queue_capacity=_capped(2 * max_slots + 256),
        run_capacity=_capped(2 * C + 64), near_horizon_us=near_horizon_us,
        meta=dict(config="gatekeeper", n_clients=C, msg_num=msg_num, junk_every=junk_every, raw=raw),
    )


# ------------------------------------------------------------- socket-state
TAG_GOT_PING_NO = 13     # socket-state/Main.hs:75-76 "Got Ping #reqNo ..."
TAG_FROM_CLIENT = 14     # "... from client #cid"


def socket_state(n_replicas: int = 1, network_delay=(ms(1), ms(5)), seed_base: int = 0,
                 max_rounds: int = 64, near_horizon_us: int = sec(20), close_every: int = 0) -> Scenario:
    """examples/socket-state/Main.hs re-hosted on the emulated transfer: a
    server counting requests per client connection with ``userStateR``
    (:65-76, :91-93), and 3 clients that send ``Ping cid`` once a second while
    ``ruskaRuletka`` (randomRIO (0,2) > 0, :96) holds, then close (:80-86).
    The server stops listening after 10 s (``invoke (after 10 sec) stop``).

    Node 0 = server, nodes 1..3 = clients, node 4 hosts main, nodes 5..7 =
    the state cells of the connections client c -> server (link c-1).  Each
    client's number of rounds is drawn host-side: draws of U[0, 2] from
    mkStdGen(seed_base + replica), client 1 first, until a 0 (capped at
    ``max_rounds``); the reference draws from the global IO generator, which is
    not reproducible.  Main holds the counts in r1..r3 (``main_regs``).

    Connections (Code.close_conn / conn_tag / conn_accept): a client tags
    each Ping with its connection number; ``close`` (MonadTransfer.hs:139-142)
    ends the connection, and the server's state cell for the link starts from
    a fresh ``mkState`` when a Ping of a newer connection arrives.  With
    ``close_every`` > 0 a client closes after every that many pings, so the
    per-connection counter restarts; the final close (:86-87) changes nothing
    observable (no later connection)."""
    SRV, SYS, STATE = 0, 4, 5
    p = Program()
    K_PING = p.kind("Ping")
    srv_set = p.listener_set({"Ping": "on_ping"})

    c = p.function("main")
    c.seti(0, SRV).fork_("server_main", node_reg=0, scratch=0)
    for cid in (1, 2, 3):
        c.mov(0, cid).seti(cid, cid)                  # r0 = rounds of client cid; node cid
        c.fork_("client_main", node_reg=cid, scratch=cid)
    c.end()

    c = p.function("server_main")
    c.listen(srv_set)                                 # stop <- listen (AtPort 4444) [...]
    c.invoke(for_(sec(10)))                           # invoke (after 10 sec) stop
    c.unlisten()
    c.end()

    c = p.function("on_ping")                         # \(Ping cid) -> do
    c.conn_accept(STATE)                              #   (the connection's socket state)
    c.user_state_load(3, 0, 1, STATE)                 #   counter <- userStateR
    c.addi(3, 1)                                      #   reqNo <- counter <+= 1
    c.user_state_store(3, 0, 1, STATE)
    c.trace(TAG_GOT_PING_NO, 3)                       #   logInfo "Got Ping #reqNo from client #cid"
    c.trace(TAG_FROM_CLIENT, 0)
    c.end()

    c = p.function("client_main")
    c.node(2)                                         # cid
    c.link(1, 0)                                      # (localhost, 4444)
    top = c.here()
    done = c.label()
    c.jeqi(0, 0, done)                                # whileM ruskaRuletka $ do
    c.wait(for_(sec(1)))                              #   wait (for 1 sec)
    c.node(2).conn_tag(2, 0, scratch=3)               #   (on the current connection)
    c.send(1, K_PING, 2)                              #   send (localhost, 4444) $ Ping cid
    c.addi(0, -1)
    if close_every:
        keep = c.label()
        c.mov(3, 0).modi(3, close_every).jnei(3, 0, keep)
        c.close_conn(0, scratch=3)                    #   close (localhost, 4444): a new socket next time
        c.bind(keep)
    c.jmp(top)
    c.bind(done)
    c.close_conn(0, scratch=3)                        # close (localhost, 4444)
    c.end()

    img = p.finalize()
    out = [[], [SRV], [SRV], [SRV], [], [], [], []]
    topo = Topology.from_out_lists(8, out)
    g = StdGenVec(seed_base + np.arange(n_replicas, dtype=np.int64))
    table = np.zeros((topo.n_links, 1, n_replicas), np.uint32)
    for l in range(topo.n_links):
        table[l, 0, :] = g.range(*network_delay)
    regs = np.zeros((n_replicas, 4), np.int64)
    for cid in (1, 2, 3):
        going = np.ones(n_replicas, bool)
        for _ in range(max_rounds):
            coin = g.range(0, 2) > 0
            going &= coin
            regs[:, cid] += going
    return Scenario(
        name="socket_state", image=img, topo=topo, n_replicas=n_replicas,
        main_pc=img.pc_of("main"), main_node=SYS, link_table=table, main_regs=regs,
        max_slots=64, queue_capacity=256, near_horizon_us=near_horizon_us,
        meta=dict(config="socket_state", seed_base=seed_base, max_rounds=max_rounds, close_every=close_every),
    )


# ------------------------------------------------------------------- gossip
TAG_RUMOR_FIRST = 9      # first receipt of the rumor at a node
K_RUMOR_PAYLOAD = 7      # forwarding is payload-independent (tie-insensitive by design)


def gossip(n_nodes: int = 1024, fanout: int = 4, n_replicas: int = 1, network_delay=(ms(1), ms(5)),
           seed: int = 0, start_us: int = sec(1), origin: int = 0, drop_log2: int = 0,
           near_horizon_us: int = sec(10), fork_strategy: str = "fork") -> Scenario:
    """Config 4: one gossip/broadcast scenario (build-defined; the reference has
    no gossip example — it composes MonadDialog `listen`/`send`, MonadDialog.hs
    :149-271, exactly like examples/ping-pong).

    Every node is a daemon already listening when the emulation starts
    (``node_listen``).  The main thread, on the origin node, waits
    ``start_us`` and sends the rumor to its ``fanout`` peers.  A node that
    receives the rumor for the first time records the time and forwards it to
    its own peers; later copies are ignored.  The forwarded payload is a
    constant, so the outcome does not depend on the order of equal-time
    deliveries.  Peers (distinct, != self) and per-link delays U[1 ms, 5 ms] are
    drawn from mkStdGen(seed); the minimum link delay (1 ms) is the lookahead
    of the node-partitioned engine.  ``fork_strategy="inline"`` runs the
    handler in place in the delivering thread (MonadDialog.hs:114-117).
    """
    if fork_strategy not in ("fork", "inline"):
        raise ValueError(f"fork_strategy must be 'fork' or 'inline', not {fork_strategy!r}")
    N, F = int(n_nodes), int(fanout)
    p = Program()
    K = p.kind("rumor")
    lset = p.listener_set({"rumor": "on_rumor"}, inline=("rumor",) if fork_strategy == "inline" else ())

    c = p.function("main")
    c.wait(for_(start_us))
    c.seti(0, K_RUMOR_PAYLOAD)
    c.nstore(0, 0)                                     # the origin knows the rumor
    c.now(3).nstore(3, 1)
    for k in range(F):
        c.link(1, k).send(1, K, 0)
    c.end()

    c = p.function("on_rumor")                        # listener: r0 = payload
    dup = c.label()
    c.nload(2, 0).jnei(2, 0, dup)                      # already seen -> ignore
    c.seti(2, 1).nstore(2, 0).now(3).nstore(3, 1)
    c.trace(TAG_RUMOR_FIRST, 0)
    for k in range(F):
        c.link(1, k).send(1, K, 0)
    c.bind(dup)
    c.end()

    img = p.finalize()
    g = StdGenVec(np.array([seed], dtype=np.int64))
    peers = np.zeros((N, F), np.int64)
    # host draw, vectorised over nodes with one generator per node (seed*N + node)
    gn = StdGenVec(np.int64(seed) * N + np.arange(N, dtype=np.int64))
    for k in range(F):
        while True:
            cand = gn.range(0, N - 2)
            cand = cand + (cand >= np.arange(N))       # skip self
            clash = np.zeros(N, bool)
            for j in range(k):
                clash |= cand == peers[:, j]
            if not clash.any() or N <= F:
                peers[:, k] = cand
                break
            # redraw only clashing nodes: keep others, loop over the mask
            peers[~clash, k] = cand[~clash]
            keep = ~clash
            while clash.any():
                c2 = gn.range(0, N - 2)
                c2 = c2 + (c2 >= np.arange(N))
                bad = np.zeros(N, bool)
                for j in range(k):
                    bad |= c2 == peers[:, j]
                take = clash & ~bad
                peers[take, k] = c2[take]
                clash &= ~take
            break
    del g
    out_off = np.arange(N + 1, dtype=np.uint32) * F
    dst = peers.reshape(-1).astype(np.uint32)
    topo = Topology(N, out_off, dst, np.full(N * F, isa.PC_NONE, np.uint32))
    gd = StdGenVec(np.int64(seed) * N + 7919 + np.arange(N, dtype=np.int64))
    table = np.zeros((N * F, 1, n_replicas), np.uint32)
    delays = np.stack([gd.range(*network_delay) for _ in range(F)], axis=1).reshape(-1).astype(np.uint32)
    if drop_log2:
        u = np.stack([gd.range(0, (1 << drop_log2) - 1) for _ in range(F)], axis=1).reshape(-1)
        delays = np.where(u == 0, delays | np.uint32(isa.LINK_DROP), delays)
    table[:, 0, :] = delays[:, None]
    listen = np.full(N, lset + 1, np.uint32)
    return Scenario(
        name=f"gossip_n{N}" + ("_inline" if fork_strategy == "inline" else ""), image=img, topo=topo, n_replicas=n_replicas,
        main_pc=img.pc_of("main"), main_node=origin, link_table=table, node_listen=listen,
        max_slots=_capped(8 * N + 64), queue_capacity=_capped(8 * N + 256), run_capacity=_capped(4 * N + 64),
        near_horizon_us=near_horizon_us,
        meta=dict(config="gossip", n_nodes=N, fanout=F, seed=seed, lookahead_us=int(network_delay[0])),
    )
