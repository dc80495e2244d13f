"""Static instruction mix of one kernel by source line and by loop (DESIGN.md 4a's ISA breakdown).

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -fopenmp -gline-tables-only --offload-device-only \\
          -c python-p2p-network_amd/csrc/relay_kernels.hip -o /tmp/rk.co
    clang-offload-bundler --unbundle --type=o --input=/tmp/rk.co \\
          --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=/tmp/rk.elf
    llvm-objdump -d -l --mcpu=gfx950 --no-show-raw-insn /tmp/rk.elf > /tmp/rk.s
    python tools/isa_lines.py /tmp/rk.s 'k_gossip_fusedILb0ELi3ELi0ELb0ELb0E' [top]

Prints the VALU / SALU / LDS counts per source line (top N) and every loop (a backward branch
and the instructions it spans) with its mix and Philox multiply count.  Static counts: a line's
dynamic weight is its trip count, which the per-round SQ counters (tools/pmc_sq.sh) bound.
"""
import collections
import re
import sys


def load(path, kernel):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^[0-9a-f]+ <.*" + kernel, l))
    base = int(lines[start].split()[0], 16)
    ins, src = [], None
    for l in lines[start + 1:]:
        if re.match(r"^[0-9a-f]+ <", l):
            break
        m = re.match(r"^; (\S+):(\d+)", l)
        if m:
            src = m.group(1).split("/")[-1] + ":" + m.group(2)
            continue
        m = re.match(r"^\t(\S+)(.*?)//\s*([0-9A-Fa-f]+):", l)
        if m:
            t = re.search(r"\+0x([0-9a-f]+)>", l)
            ins.append((int(m.group(3), 16), m.group(1), base + int(t.group(1), 16) if t else None, src))
    return ins


def kind(op):
    return "v" if op.startswith("v_") else "s" if op.startswith("s_") else "ds" if op.startswith("ds_") else "mem"


def main():
    path, kernel = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    ins = load(path, kernel)
    print(f"{len(ins)} instructions;", dict(collections.Counter(kind(op) for _, op, _, _ in ins)))
    per = collections.defaultdict(collections.Counter)
    for _, op, _, src in ins:
        per[src][kind(op)] += 1
    for src, c in sorted(per.items(), key=lambda x: -x[1]["v"])[:top]:
        print(f"  {src}: VALU {c['v']} SALU {c['s']} LDS {c['ds']} mem {c['mem']}")
    idx = {a: i for i, (a, _, _, _) in enumerate(ins)}
    print("loops (backward branches):")
    for i, (a, op, tgt, _) in enumerate(ins):
        if (op.startswith("s_cbranch") or op == "s_branch") and tgt is not None and tgt <= a and tgt in idx:
            body = ins[idx[tgt]:i + 1]
            c = collections.Counter(kind(x[1]) for x in body)
            mads = sum(1 for x in body if x[1] == "v_mad_u64_u32")
            print(f"  [{idx[tgt]}, {i}] {len(body)} instructions {dict(c)} v_mad_u64_u32 {mads} from {body[0][3]}")


if __name__ == "__main__":
    main()
