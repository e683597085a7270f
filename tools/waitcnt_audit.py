"""Static audit of the event kernels' compiled code (hipcc -S of engine.hip).

For every tw_run_kernel instantiation:

1. pass-head waits: the vector-memory waits at the head of the interpreter
   pass loop and right after the record prefetch.  A vmcnt wait there means
   some path leaves a load in flight into the step, so the compiler waits for
   everything outstanding (the prefetch, the previous pass's stores) on every
   pass -- the prefetch then no longer overlaps the step (a performance
   finding, reported).

2. counted waits (a correctness check, the exit status): the record prefetch
   and the far-run prefetch are LDS-DMA loads (`global_load_lds_dwordx4`,
   inline asm the compiler's wait-count pass does not model), and the code
   that reads what they wrote proves they landed with a hand-counted
   `s_waitcnt vmcnt(N)` (engine_dev.hpp: Lane::fetch_rec TW_TAIL_VMEM,
   run_commit, the LP child staging): N is the number of vector-memory
   instructions the code issues after the load it guards.  Loads and waits
   carry a `; tw:<stream>` comment (pf: the record prefetch, run: a far run's
   next entry, vic: the throwTo victims' header quads staged at the pop).  A dataflow pass over the kernel's control-flow graph computes,
   per stream, at every such wait, the FEWEST vector-memory instructions issued
   since that stream's most recent LDS-DMA load on any path reaching it (a wait
   that already covered the load ends the concern).  If that count is below N
   on some path, vmcnt(N) would not prove the load landed and the code could
   read stale LDS staging: a violation.

usage: python tools/waitcnt_audit.py <engine.s>   (exit 1 on a violation)
"""
import re
import sys

INF = 1 << 30
VMEM = re.compile(r"^\s*(global_|buffer_|flat_|scratch_)")
LDS_DMA = re.compile(r"^\s*global_load_lds_")
WAIT = re.compile(r"^\s*s_waitcnt\b(.*)$")
VMCNT = re.compile(r"vmcnt\((\d+)\)")
LABEL = re.compile(r"^(\.LBB\w+|\.Ltmp\w+):")
BRANCH = re.compile(r"^\s*(s_branch|s_cbranch_\w+)\s+(\.LBB\w+)")


def blocks_of(body):
    """Basic blocks: (label, [instruction lines], successor labels)."""
    blocks = []
    cur = {"label": "__entry__", "ins": [], "succ": [], "fall": True}
    n = 0
    for line in body:
        m = LABEL.match(line)
        if m:
            blocks.append(cur)
            cur = {"label": m.group(1), "ins": [], "succ": [], "fall": True}
            continue
        s = line.split(";")[0].rstrip() if not line.strip().startswith(";;#ASM") else line.strip()
        t = re.search(r";\s*tw:\w+", line)
        if t and s.strip():
            s = s + " " + t.group(0)  # (keep the stream tag of an LDS-DMA load or counted wait)
        if not s.strip():
            if ";;#ASMSTART" in line or ";;#ASMEND" in line:
                cur["ins"].append(line.strip())
            continue
        cur["ins"].append(s.strip())
        b = BRANCH.match(s)
        if b:
            # a block ends at every branch: its target sees the value here
            cur["succ"].append(b.group(2))
            cur["fall"] = b.group(1) != "s_branch"
            blocks.append(cur)
            n += 1
            cur = {"label": f"__anon{n}__", "ins": [], "succ": [], "fall": True}
        elif s.strip().startswith("s_endpgm") or s.strip().startswith("s_setpc_b64"):
            cur["fall"] = False
            blocks.append(cur)
            n += 1
            cur = {"label": f"__anon{n}__", "ins": [], "succ": [], "fall": True}
    blocks.append(cur)
    for i, b in enumerate(blocks):
        if b["fall"] and i + 1 < len(blocks):
            b["succ"].append(blocks[i + 1]["label"])
    return blocks


TAG = re.compile(r";\s*tw:(\w+)")
STREAMS = ("pf", "run", "vic")


def transfer(ins, v, checks=None):
    """v[stream]: vector-memory instructions issued since that stream's last
    LDS-DMA load that no wait has covered yet (INF: none outstanding)."""
    v = dict(v)
    for s in ins:
        if s.startswith(";;#ASM"):
            continue
        tag = TAG.search(s)
        if LDS_DMA.match(s):
            for t in STREAMS:  # every outstanding load has one more younger op
                v[t] = v[t] + 1 if v[t] < INF else INF
            if tag:
                v[tag.group(1)] = 0
            continue
        if VMEM.match(s):
            for t in STREAMS:
                v[t] = v[t] + 1 if v[t] < INF else INF
            continue
        w = WAIT.match(s)
        if w:
            m = VMCNT.search(w.group(1))
            if not m:
                continue
            k = int(m.group(1))
            if tag and checks is not None and v[tag.group(1)] < INF:
                checks.append((s, k, v[tag.group(1)]))
            for t in STREAMS:
                if v[t] < INF and v[t] >= k:
                    v[t] = INF  # that stream's load has landed
    return v


def counted_waits(body):
    bl = blocks_of(body)
    idx = {b["label"]: i for i, b in enumerate(bl)}
    inv = [None] * len(bl)  # value at block entry (None: not reached yet)
    inv[0] = {t: INF for t in STREAMS}
    work = [0]
    while work:
        i = work.pop()
        out = transfer(bl[i]["ins"], inv[i])
        for lab in bl[i]["succ"]:
            j = idx.get(lab)
            if j is None:
                continue
            nv = out if inv[j] is None else {t: min(inv[j][t], out[t]) for t in STREAMS}
            if nv != inv[j]:
                inv[j] = nv
                work.append(j)
    checks = []
    for i, b in enumerate(bl):
        if inv[i] is not None:
            transfer(b["ins"], inv[i], checks)
    # counted waits the walk reached at all (with or without a load in flight)
    reached = sum(1 for i, b in enumerate(bl) if inv[i] is not None
                  for x in b["ins"] if WAIT.match(x) and TAG.search(x))
    return checks, reached


def main():
    s = open(sys.argv[1]).read().split("\n")
    if not any(TAG.search(l) for l in s):
        print("no tagged LDS-DMA loads (a TW_DMA_BUILTIN build?): nothing to check")
        return 1
    starts = [(i, m.group(1)) for i, l in enumerate(s) if (m := re.match(r"(_ZN12_GLOBAL__N_113tw_run_kernel\S+):", l))]
    slow = bad = 0
    for i0, name in starts:
        end = next(i for i in range(i0, len(s)) if s[i].strip().startswith(".size") and name in s[i])
        raw = s[i0 + 1:end]
        body = [l for l in raw if "implicit-def" not in l]
        ffs = [i for i, l in enumerate(body) if "s_ff1_i32_b64" in l]
        idx = [i for i, l in enumerate(body) if "global_load_lds_dwordx4" in l]
        head = [l.strip() for l in body[ffs[0] - 15:ffs[0] + 25] if "vmcnt" in l] if ffs else []
        pf = [l.strip() for l in body[idx[-1]:idx[-1] + 40] if "vmcnt" in l] if idx else []
        slow += bool(head or pf)
        tag = re.search(r"kernelI(.*)EEvN2tw", name).group(1)
        checks, reached = counted_waits(raw)
        viol = [(w, k, v) for w, k, v in checks if v < k]
        bad += bool(viol)
        kinds = sorted({k for _, k, _ in checks})
        if idx and not reached:
            viol = [("(no counted wait reached at all: the audit lost the kernel's paths)", 1, 0)]
            bad += 1
        print(f"{tag:40s} pass-head vmcnt: {head or '-'}  after-prefetch vmcnt: {pf or '-'}  "
              f"counted waits vmcnt{kinds}: {len(checks)} reached with a prefetch in flight, "
              f"{len(viol)} short")
        for w, k, v in viol[:8]:
            print(f"    SHORT: `{w}` reached after only {v} vector-memory ops since an LDS-DMA load")
    print("kernels with a pass-head / after-prefetch wait:", slow)
    print("kernels with a short counted wait:", bad)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
