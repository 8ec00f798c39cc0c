"""VGPRs / spills / scratch of every k_chain_run instance (hipcc -Rpass-analysis=kernel-resource-usage).
   python tools/kernel_regs.py [source.hip]   (default: the chain kernels)"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "mcmc-in-tonga_amd", "csrc", "chain_kernels.hip")
flags = "-O3 -std=c++17 -ffp-contract=off -fno-fast-math -Wno-unused-result --offload-arch=gfx950 -munsafe-fp-atomics"
p = subprocess.run(["/opt/rocm/bin/hipcc"] + flags.split() + sys.argv[2:] + ["-c", src, "-o", "/tmp/kernel_regs.o",
                    "-Rpass-analysis=kernel-resource-usage"], cwd=os.path.dirname(src), capture_output=True, text=True)
cur = None
rows = {}
for line in p.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|VGPRs Spill|SGPRs Spill|ScratchSize \[bytes/lane\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1)] = int(m.group(2))
for name, r in rows.items():
    m = re.search(r"k_chain_runILb(\d)ELb(\d)ELi(\d+)ELb(\d)ELb(\d)E", name)
    if not m:
        continue
    print("k_chain_run<SMALL=%s SCRIPT=%s NTH=%s RLDS=%s ROUNDS=%s>: VGPR %d, VGPR spill %d, SGPR spill %d, scratch %d" % (
        m.group(1), m.group(2), m.group(3), m.group(4), m.group(5), r.get("VGPRs", -1), r.get("VGPRs Spill", -1),
        r.get("SGPRs Spill", -1), r.get("ScratchSize [bytes/lane]", -1)))
