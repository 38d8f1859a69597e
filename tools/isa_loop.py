"""Instruction counts of a kernel's inner loop in a hipcc -S listing (measurement aid):

    hipcc --offload-arch=gfx950 ... --cuda-device-only -S -o render.s langsplat_amd/csrc/lsr_render.hip
    python3 tools/isa_loop.py render.s k_render_forwardILb0ELb1ELb1E "ds_read_b96"

Finds the kernel's loops (labels marked "Loop Header" by the compiler) whose first 25 lines contain
the marker, and prints the VALU / SALU / s_waitcnt / LDS counts between the header and the last
branch back to it (every block of the loop body, whichever path a wave takes).
"""
import re
import sys


def main():
    path, kernel, marker = sys.argv[1], sys.argv[2], sys.argv[3]
    lines = open(path).read().split("\n")
    start = next(k for k, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(kernel) + r"\S*:", l))
    end = next(k for k in range(start, len(lines)) if lines[k].startswith(".Lfunc_end"))
    b = lines[start:end]
    # blocks: (label, annotation, lines); the compiler marks each block of a loop with
    # "in Loop: Header=BBx_y Depth=d" (the header itself: "Loop Header")
    blocks, cur = [], None
    for l in b:
        m = re.match(r"^(\.LBB\S+|; %bb\.\d+):?(.*)$", l)
        if m:
            cur = [m.group(1).lstrip("; %").rstrip(":"), m.group(2), []]
            blocks.append(cur)
        elif cur is not None:
            if l.strip().startswith(";"):
                cur[1] += l
            else:
                cur[2].append(l.strip())
    for lab, ann, _ in blocks:
        if "Loop Header" not in ann or not lab.startswith(".LBB"):
            continue
        h = lab[2:]  # BBx_y
        body = [x for lb, an, ls in blocks if lb == lab or re.search(r"Header=" + re.escape(h) + r"\b", an) for x in ls]
        if not any(marker in x for x in body):
            continue
        ins = [x for x in body if x and not x.startswith(".")]
        v = sum(x.startswith("v_") for x in ins)
        w = sum(x.startswith("s_waitcnt") for x in ins)
        nop = sum(x.startswith("s_nop") for x in ins)
        sc = sum(x.startswith("s_") for x in ins) - w - nop
        ds = sum(x.startswith("ds_") for x in ins)
        print(f"{lab}: VALU {v}  SALU {sc}  s_nop {nop}  s_waitcnt {w}  LDS {ds}")

if __name__ == "__main__":
    main()
