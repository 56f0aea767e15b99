"""Per-kernel register / LDS / occupancy of a HIP source as the compiler
reports it (-Rpass-analysis=kernel-resource-usage), plus the workgroups per
CU that the SGPR residency rule of MI355X_MICROARCH.md admits
(min(8, floor(800 / (ceil(sgpr/16)*16 + 16))) waves per SIMD).

Usage: python tools/kernel_resources.py etcd_amd/csrc/qb_tracker_bucket.hip [regex] [-D...]
"""
import re
import subprocess
import sys
import tempfile

src = sys.argv[1]
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else None
defs = [a for a in sys.argv[2:] if a.startswith("-D")]
with tempfile.NamedTemporaryFile(suffix=".o") as o:
    out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                          "-Iinclude", "-Ietcd_amd/csrc", "-munsafe-fp-atomics", *defs, "-x", "hip",
                          "-c", src, "-o", o.name, "-Rpass-analysis=kernel-resource-usage"],
                         capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?): (.*?) \[", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
dem = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                     text=True).stdout.splitlines()
for r, d in zip(rows, dem):
    if pat and not pat.search(d):
        continue
    sg = int(r.get("TotalSGPRs", 0))
    w_sgpr = min(8, 800 // ((sg + 15) // 16 * 16 + 16))
    print(f"{d[:90]:90s} sgpr {sg:3d} (<= {w_sgpr} w/SIMD) vgpr {r.get('VGPRs'):>3s} "
          f"occ {r.get('Occupancy [waves/SIMD]')} lds {r.get('LDS Size [bytes/block]')} "
          f"spill s{r.get('SGPRs Spill')} v{r.get('VGPRs Spill')}")
