"""Register / spill summary of the policy and update kernels (compile only, no GPU):

    python tools/kres.py [extra hipcc flags, e.g. -DSHIPENV_X3P=0]
"""
import re
import subprocess
import sys

cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
       "--offload-arch=gfx950", "--cuda-device-only", "-S", "-o", "/tmp/kres.s",
       "shippingenv_amd/csrc/shipenv.hip", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[1:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|SGPRs Spill|VGPRs Spill): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split(" [")[0]] = int(m.group(2))
for k, v in rows.items():
    if "policy" in k or "qtrain" in k:
        name = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", k)[:60]
        print(f"{name:60s} vgpr {v.get('VGPRs')} sgpr {v.get('TotalSGPRs')} vspill {v.get('VGPRs Spill')} "
              f"sspill {v.get('SGPRs Spill')} scratch {v.get('ScratchSize')} waves {v.get('Occupancy')}")
