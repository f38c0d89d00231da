"""Summarise hipcc `-Rpass-analysis=kernel-resource-usage` remarks (one line per kernel: VGPRs,
AGPRs, occupancy, scratch, VGPR spills), e.g. to check that no conv tile spills after a change:

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -c csrc/kernels/conv_igemm_g0.hip -Icsrc/kernels \\
        -o /tmp/g0.o -Rpass-analysis=kernel-resource-usage 2> /tmp/g0.txt
    python tools/kernel_resources.py /tmp/g0.txt [--spills]
"""
import re
import sys

KEYS = {"VGPRs": "v", "AGPRs": "a", "Occupancy [waves/SIMD]": "occ", "ScratchSize [bytes/lane]": "scratch",
        "VGPRs Spill": "vspill", "SGPRs Spill": "sspill"}


def parse(paths):
    rows = []
    for p in paths:
        cur = None
        for line in open(p):
            m = re.search(r"Function Name: (\S+)", line)
            if m:
                cur = {"name": m.group(1)}
                rows.append(cur)
                continue
            if cur is None:
                continue
            for k, short in KEYS.items():
                m = re.search(r"remark:\s+" + re.escape(k) + r": (\d+)", line)
                if m:
                    cur[short] = int(m.group(1))
    return rows


def short_name(n):
    m = re.search(r"conv_igemm_kernelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELb(\d)E(\w)Li(\d)ELi(\d)E", n)
    return "conv_igemm<%s>" % ",".join(m.groups()) if m else n[:70]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    rows = parse(args)
    for r in rows:
        if "--spills" in sys.argv and not (r.get("vspill") or r.get("scratch")):
            continue
        print(f"{short_name(r['name']):48s} v {r.get('v')} a {r.get('a')} occ {r.get('occ')} "
              f"scratch {r.get('scratch')} vspill {r.get('vspill')} sspill {r.get('sspill')}")


if __name__ == "__main__":
    main()
