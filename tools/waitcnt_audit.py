"""Static audit of the event kernels' compiled code (hipcc -S of engine.hip):
for every tw_run_kernel instantiation, the vector-memory waits at the head of
the interpreter pass loop and right after the record prefetch.  A vmcnt wait
there means some path leaves a load in flight into the step, so the compiler
waits for everything outstanding (the prefetch, the previous pass's stores)
on every pass -- the prefetch then no longer overlaps the step.

usage: python tools/waitcnt_audit.py <engine.s>
"""
import re
import sys


def main():
    s = open(sys.argv[1]).read().split("\n")
    starts = [(i, m.group(1)) for i, l in enumerate(s) if (m := re.match(r"(_ZN12_GLOBAL__N_113tw_run_kernel\S+):", l))]
    bad = 0
    for i0, name in starts:
        end = next(i for i in range(i0, len(s)) if s[i].strip().startswith(".size") and name in s[i])
        body = [l for l in s[i0:end] if "implicit-def" not in l]
        ffs = [i for i, l in enumerate(body) if "s_ff1_i32_b64" in l]
        idx = [i for i, l in enumerate(body) if "global_load_lds_dwordx4" in l]
        head = [l.strip() for l in body[ffs[0] - 15:ffs[0] + 25] if "vmcnt" in l] if ffs else []
        pf = [l.strip() for l in body[idx[-1]:idx[-1] + 40] if "vmcnt" in l] if idx else []
        bad += bool(head or pf)
        tag = re.search(r"kernelI(.*)EEvN2tw", name).group(1)
        print(f"{tag:40s} pass-head vmcnt: {head or '-'}  after-prefetch vmcnt: {pf or '-'}")
    print("kernels with a wait:", bad)


if __name__ == "__main__":
    main()
