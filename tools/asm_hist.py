"""Instruction histogram of one kernel in a hipcc -S listing, per basic block:
    python tools/asm_hist.py <file.s> <kernel-name-substring> [min-block-size]"""
import collections
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    minsz = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(pat) or (pat in l and l.endswith(pat + ":")) or
                 (l.split(":")[0].find(pat) >= 0 and not l.startswith(("\t", " ", ";", "."))))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur, name = [], collections.Counter(), "entry"
    for l in lines[start + 1:end]:
        t = l.strip()
        if t.endswith(":") and not t.startswith(";"):
            blocks.append((name, cur))
            name, cur = t[:-1], collections.Counter()
            continue
        if not t or t.startswith((".", ";")):
            continue
        cur[t.split()[0]] += 1
    blocks.append((name, cur))
    tot = collections.Counter()
    for n, c in blocks:
        tot.update(c)
        s = sum(c.values())
        if s >= minsz:
            valu = sum(v for k, v in c.items() if k.startswith("v_") and "mfma" not in k)
            print(f"{n}: {s} instr, {valu} VALU, {c.get('v_mfma_i32_16x16x64_i8', 0) + c.get('v_mfma_f32_16x16x32_bf16', 0)} MFMA")
            for k, v in c.most_common(25):
                print(f"    {v:6d} {k}")
    print("total", sum(tot.values()))


if __name__ == "__main__":
    main()
