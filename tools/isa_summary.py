"""Per-function size, scratch traffic, calls and barriers of a disassembled code object (llvm-objdump -d)."""
import re
import sys
from collections import Counter

lines = open(sys.argv[1]).read().splitlines()
name, funcs = None, {}
for l in lines:
    m = re.match(r'^([0-9a-f]+) <(.*)>:', l)
    if m:
        name = m.group(2)
        funcs[name] = []
        continue
    m = re.match(r'^\s+([a-z_0-9]+)\s.*//\s*([0-9A-F]+):', l)
    if name and m:
        funcs[name].append((int(m.group(2), 16), m.group(1)))
sel = sys.argv[2] if len(sys.argv) > 2 else ""
for n, ins in funcs.items():
    if sel not in n or not ins:
        continue
    c = Counter(op for _, op in ins)
    sc = sum(v for k, v in c.items() if k.startswith("scratch") or k.startswith("buffer_"))
    print("%-90s %6d ins %6.1f KB scratch %4d calls %3d barriers %3d memtime %3d" % (
        n[:90], len(ins), (ins[-1][0] - ins[0][0]) / 1024, sc, c["s_swappc_b64"], c["s_barrier"], c["s_memtime"]))
