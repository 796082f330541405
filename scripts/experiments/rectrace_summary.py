"""Summarise k_rec_g phase timestamps (rectrace_rg8.txt / rectrace_rg16.txt in DIR).
    python scripts/experiments/rectrace_summary.py DIR"""
import numpy as np, sys
for g in (8, 16):
    a = np.loadtxt(f"{sys.argv[1]}/rectrace_rg{g}.txt", dtype=np.int64)
    wg, t0, t1, t2, t3, hw = a.T
    base = t0.min()
    ns = lambda x: (x - base) * 10  # 100 MHz -> ns
    nsw8 = 56
    ps = wg < nsw8; pb = ~ps
    print(f"RG={g}: {len(a)} workgroups ({ps.sum()} pair-scalar, {pb.sum()} pair-block)")
    print(f"  start spread: pair-scalar {ns(t0[ps]).min()/1e3:.2f}-{ns(t0[ps]).max()/1e3:.2f} us, pair-block {ns(t0[pb]).min()/1e3:.2f}-{ns(t0[pb]).max()/1e3:.2f} us")
    print(f"  last end: {ns(t3).max()/1e3:.2f} us; pair-scalar end max {ns(t3[ps]).max()/1e3:.2f} us")
    d = lambda x, y: (y[pb] - x[pb]) * 10 / 1e3
    for name, x, y in (("start->staged", t0, t1), ("staged->loop done", t1, t2), ("loop->end(epilogue)", t2, t3), ("total", t0, t3)):
        v = d(x, y); print(f"  {name:22s} median {np.median(v):6.2f} us  p10 {np.percentile(v,10):6.2f}  p90 {np.percentile(v,90):6.2f}  max {v.max():6.2f}")
    ends = np.sort(ns(t3[pb]))/1e3
    print(f"  pair-block ends: 50% by {ends[len(ends)//2]:.2f} us, 90% by {ends[int(.9*len(ends))]:.2f} us, last {ends[-1]:.2f}")
    # CU id from HW_ID: bits: wave_id[3:0], simd_id[5:4], pipe_id[7:6], cu_id[11:8], sh_id[12], se_id[15:13] (gfx9)
    cu = (hw >> 8) & 0xF; se = (hw >> 13) & 0x7; sh = (hw >> 12) & 1
    key = se * 32 + sh * 16 + cu
    print(f"  distinct (se,sh,cu) slots seen: {len(set(key.tolist()))}")
