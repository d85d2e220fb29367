"""Summarise `hipcc -Rpass-analysis=kernel-resource-usage` output per pass kernel (P, T)."""
import re
import sys

txt = open(sys.argv[1]).read()
tmin = int(sys.argv[2]) if len(sys.argv) > 2 else 0
OCC = r"Occupancy \[waves/SIMD\]"
for p in re.split(r"remark: Function Name: ", txt)[1:]:
    name = p.split()[0]
    m = re.match(r"_ZN4rs1611pass_kernelILi(\d+)ELi(\d+)E", name)
    if not m or int(m.group(2)) < tmin:
        continue

    def g(k):
        mm = re.search(k + r": (\d+)", p)
        return mm.group(1) if mm else "?"

    print("P%s T%s  VGPR %s  SGPR %s  occ %s  sspill %s  vspill %s" % (
        m.group(1), m.group(2), g("VGPRs"), g("SGPRs"), g(OCC), g("SGPRs Spill"), g("VGPRs Spill")))
