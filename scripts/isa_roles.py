"""Instructions of one loop of a kernel's ISA, by role (count the decompress
walker's instructions per bin by role).  Input: device assembly with line tables, e.g.

  hipcc --offload-arch=gfx950 -O3 -std=c++17 -g -fPIC --cuda-device-only -S \\
      avrecode_amd/csrc/avr_k_decompress.hip -o /tmp/dec_g.s
  python scripts/isa_roles.py /tmp/dec_g.s 'slices_parallel_kernelILi1ELb0ELb0E' --anchor 1562 1596
  python scripts/isa_roles.py /tmp/dec_g.s 'slices_parallel_kernelILi1ELb0ELb0E' --loop 4887

Each instruction carries the inlining chain of its .loc comment; its role is the first frame of the
chain that falls in a known range of avr_walker.h / avr_engine.h (ROLES below).  --anchor LINE CALLER
lists the innermost loops holding an instruction inlined from LINE through CALLER; --loop HDR prints
that loop's blocks (not those of loops nested in it) with their roles and the per-role sums.  The
code generation only: which blocks a bin runs is read off the listing."""
import argparse
import collections
import re
import sys

W, E = "avr_walker.h", "avr_engine.h"
# (file, first line, last line, role): the decompress walker's map, level and bin helpers
ROLES = [
    (E, 392, 396, "est_update"), (E, 535, 573, "decision"), (E, 60, 110, "decision"),
    (W, 562, 591, "est_lookup"), (W, 609, 620, "est_lookup"),
    (W, 592, 605, "est_store"), (W, 1562, 1567, "est_store"), (W, 1585, 1588, "est_store"),
    (W, 912, 933, "decision"), (W, 935, 950, "decision"), (W, 420, 425, "decision"),
    (W, 432, 500, "op_emit"), (W, 258, 275, "op_emit"), (W, 960, 979, "op_emit"),
    (W, 1569, 1570, "op_emit"), (W, 1578, 1583, "op_emit"), (W, 1589, 1592, "op_emit"), (W, 1658, 1660, "op_emit"),
    (W, 1545, 1557, "context"), (W, 1649, 1649, "context"), (W, 1653, 1653, "context"),
    (W, 1544, 1544, "bookkeeping"), (W, 1568, 1568, "bookkeeping"), (W, 1571, 1577, "bookkeeping"),
    (W, 1647, 1647, "bookkeeping"), (W, 1650, 1657, "bookkeeping"), (W, 1668, 1669, "bookkeeping"),
    (W, 354, 360, "sync"),
]


def role(chain):
    for f, l in chain:
        for rf, a, b, r in ROLES:
            if f == rf and a <= l <= b:
                return r
    return "control"   # branches, joins and moves the line table gives to no helper (line 0)


def parse(path, kernel):
    blocks, cur, chain, on = [], None, (), False
    for line in open(path):
        s = line.strip()
        if not on:
            on = s.startswith("_ZN") and ":" in s and kernel in s.split(":")[0]   # the kernel's label
            continue
        if s.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):(.*)$", s)
        if m:
            lab = m.group(1).replace("; ", "")
            cur = {"label": lab, "id": re.split(r"[_.]", lab)[-1], "hdr": None, "ins": []}
            blocks.append(cur)
            mm = re.search(r"Header=BB\d+_(\d+)", m.group(2))
            if mm:
                cur["hdr"] = mm.group(1)
            continue
        if s.startswith(";") and cur is not None and not cur["ins"]:
            if "Loop Header" in s:
                cur["hdr"] = cur["id"]
            elif "in Loop:" in s:
                mm = re.search(r"Header=BB\d+_(\d+)", s)
                if mm:
                    cur["hdr"] = mm.group(1)
            continue
        if s.startswith(".loc"):
            c = s.split(";", 1)[1] if ";" in s else ""
            chain = tuple((a.split("/")[-1], int(b)) for a, b in re.findall(r"csrc/([\w./]+):(\d+):\d+", c))
            continue
        if not s or s.startswith(".") or s.startswith(";") or cur is None:
            continue
        cur["ins"].append((s.split()[0], chain))
    return blocks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--anchor", type=int, nargs=2)
    ap.add_argument("--loop")
    a = ap.parse_args()
    blocks = parse(a.asm, a.kernel)
    print(f"{len(blocks)} blocks, {sum(len(b['ins']) for b in blocks)} instructions", file=sys.stderr)
    if a.anchor:
        line, caller = a.anchor
        hits = collections.Counter()
        for b in blocks:
            for _, ch in b["ins"]:
                ls = [l for f, l in ch if f == W]
                if line in ls and caller in ls:
                    hits[b["hdr"]] += 1
                    break
        for h, n in hits.most_common():
            print(f"loop {h}: {n} blocks with the anchor")
    if a.loop:
        tot = collections.Counter()
        for b in blocks:
            if b["hdr"] != a.loop:
                continue
            c = collections.Counter(role(ch) for _, ch in b["ins"])
            tot.update(c)
            print(f"{b['label']:14s} {len(b['ins']):3d}  " + " ".join(mn for mn, _ in b["ins"]))
            print(" " * 20 + ", ".join(f"{k} {v}" for k, v in c.most_common()))
        print("loop total:", dict(tot.most_common()))


if __name__ == "__main__":
    main()
