"""Per-kernel register / scratch / occupancy table from hipcc's
`-Rpass-analysis=kernel-resource-usage` remarks (make -C time-warp_amd resource-usage).

usage: make -s -C time-warp_amd resource-usage 2>&1 | python tools/resource_usage.py [--scratch-only]
"""
import re
import sys

KEYS = {"VGPRs": "vgpr", "AGPRs": "agpr", "ScratchSize [bytes/lane]": "scratch", "SGPRs Spill": "sspill",
        "VGPRs Spill": "vspill", "Occupancy [waves/SIMD]": "occ", "LDS Size [bytes/block]": "lds"}


def parse(lines):
    out, cur = [], None
    for line in lines:
        m = re.search(r"remark: (Function Name|[A-Za-z ]+(?:\[[^\]]*\])?): (\S+)", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2)
        if k == "Function Name":
            cur = {"name": v}
            out.append(cur)
        elif cur is not None and k in KEYS:
            cur[KEYS[k]] = int(v)
    return out


def short(name):
    m = re.search(r"(tw_\w+?kernel|tw_\w+)I(.*)E(?:E|Ev)", name)
    if not m:
        return name[:60]
    args = re.findall(r"L([bi])(\d+)E", m.group(2))
    return m.group(1) + "<" + ",".join(("true" if v == "1" else "false") if t == "b" else v for t, v in args) + ">"


def main():
    rows = parse(sys.stdin)
    only = "--scratch-only" in sys.argv
    print(f"{'kernel':58s} {'vgpr':>4s} {'agpr':>4s} {'scr':>4s} {'sspl':>4s} {'vspl':>4s} {'occ':>3s} {'lds':>6s}")
    for r in rows:
        if only and not r.get("scratch"):
            continue
        print(f"{short(r['name']):58s} {r.get('vgpr', 0):4d} {r.get('agpr', 0):4d} {r.get('scratch', 0):4d} "
              f"{r.get('sspill', 0):4d} {r.get('vspill', 0):4d} {r.get('occ', 0):3d} {r.get('lds', 0):6d}")


if __name__ == "__main__":
    main()
