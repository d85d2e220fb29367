"""Compile rs16_kernels.hip with -Rpass-analysis=kernel-resource-usage and
print one line per kernel: VGPRs, SGPRs, spills, scratch, occupancy."""
import re, subprocess, sys
src = sys.argv[1] if len(sys.argv) > 1 else "reed-solomon-16_amd/csrc/rs16_kernels.hip"
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", src, "-o", "/tmp/kstats.o",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None; rows = {}
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
    if not m: 
        if "error" in line: print(line)
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip(); rows[cur] = {}
    elif cur and ":" in t:
        k, v = t.split(":", 1); rows[cur][k.strip()] = v.strip()
def short(n):
    m = re.match(r"_ZN4rs1611pass_kernelILi(\d+)ELi(\d+)E", n)
    return f"pass<{m.group(1)},{m.group(2)}>" if m else n[:40]
print(f"{'kernel':44s} {'VGPR':>5} {'SGPR':>5} {'sSpl':>5} {'vSpl':>5} {'scr':>5} {'occ':>4}")
for n, r in rows.items():
    s = short(n)
    if flt and flt not in s: continue
    print(f"{s:44s} {r.get('VGPRs','?'):>5} {r.get('TotalSGPRs','?'):>5} {r.get('SGPRs Spill','?'):>5} {r.get('VGPRs Spill','?'):>5} {r.get('ScratchSize [bytes/lane]','?'):>5} {r.get('Occupancy [waves/SIMD]','?'):>4}")
