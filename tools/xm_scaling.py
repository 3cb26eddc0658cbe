"""Per-launch rate of the band-reduction streaming kernels against the
trailing size m, from a rocprofv3 kernel trace of one solve (development
tool): m is recovered from the launch order (each X/M launch is one panel,
m = n - 32 (p + 1); pairs: one update per two panels).
    python tools/xm_scaling.py run_kernel_trace.csv N"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2])
# the last solve: from the last bulge launch backwards to the previous one
bul = [i for i, r in enumerate(rows) if "bulge" in r["Kernel_Name"]]
lo = bul[-2] + 1 if len(bul) > 1 else 0
rs = rows[lo:bul[-1]]


def dur(r):
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3


for pat, label in (("xm_kernel", "X/M"), ("syr2k_w", "update"), ("pqr_kernel", "panel QR")):
    ks = [r for r in rs if pat in r["Kernel_Name"]]
    print(f"{label}: {len(ks)} launches, {sum(map(dur, ks)) / 1e3:.2f} ms")
    step = max(1, len(ks) // 12)
    for i in range(0, len(ks), step):
        r = ks[i]
        frac = i / max(len(ks), 1)
        m = int(n * (1 - frac))
        gb = 8.0 * m * m / 1e9
        print(f"   #{i:4d} m~{m:6d} {dur(r):8.1f} us  {re.sub(r'[(].*', '', r['Kernel_Name'])[:40]:40s}"
              f"  A22 {gb:6.3f} GB -> {gb / (dur(r) * 1e-6) / 1e3:5.2f} TB/s")
