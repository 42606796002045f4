"""Per-kernel register / scratch / occupancy / LDS table of kernels.hip for
gfx950 (compiler remarks).  Dev tool: `python3 kres.py` from this directory."""
import re
import subprocess

cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
       "-fno-fast-math", "-I../../include", "-c", "kernels.hip", "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        name = t.split(":", 1)[1].strip()
        cur = None
        if "rocprim" in name:
            continue
        name = re.sub(r"_ZN3otm12_GLOBAL__N_1\d+", "", name)
        name = re.sub(r"ENS_\d.*|EPK.*|EvNS_.*", "", name)
        cur = {"name": name}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    print("%-34s vgpr %4s agpr %4s scratch %4s occ %2s lds %6s" % (
        r["name"][:34], r.get("VGPRs"), r.get("AGPRs"), r.get("ScratchSize [bytes/lane]"),
        r.get("Occupancy [waves/SIMD]"), r.get("LDS Size [bytes/block]")))
