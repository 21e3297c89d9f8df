"""Instruction mix of kernels in a device assembly file (hipcc --cuda-device-only -S).

usage: asm_mix.py FILE.s SUBSTRING [SUBSTRING ...]   -- every function whose demangled name
contains all substrings: instruction counts by mnemonic (top 40) and the loop bodies' sizes."""
import re
import subprocess
import sys
from collections import Counter


def functions(path):
    s = open(path).read()
    for m in re.finditer(r'^(_Z\w+):[^\n]*\n(.*?)^\.Lfunc_end\d+:', s, re.S | re.M):
        yield m.group(1), m.group(2)


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    for name, body in functions(path):
        dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        if not all(x in dm for x in subs):
            continue
        ins = [l.strip() for l in body.split("\n") if l.startswith("\t") and not l.strip().startswith((".", ";"))]
        c = Counter(i.split()[0] for i in ins)
        print(dm[:160])
        print("  total", len(ins), "  " + " ".join(f"{k}:{v}" for k, v in c.most_common(40)))


if __name__ == "__main__":
    main()
