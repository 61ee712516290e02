"""Instruction histogram of one kernel in a gfx950 .s file (hipcc -S
--offload-device-only).  Usage: python tools/isa_hist.py file.s kernel_substr [top]"""
import collections
import sys


def kernel_body(lines, name):
    start = None
    for i, l in enumerate(lines):
        if start is None and l.startswith("_Z") and name in l.split(":")[0]:
            start = i
        elif start is not None and "s_endpgm" in l:
            return lines[start:i + 1]
    raise SystemExit(f"kernel {name} not found")


def main():
    lines = open(sys.argv[1]).read().split("\n")
    body = kernel_body(lines, sys.argv[2])
    ins = []
    for l in body:
        t = l.strip()
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        ins.append(t.split()[0])
    c = collections.Counter(ins)
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    print(f"total {len(ins)}  valu {valu}")
    for k, v in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 30):
        print(f"{v:7d} {k}")


if __name__ == "__main__":
    main()
