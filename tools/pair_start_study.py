"""Oracle study (CPU, development): per taxon and model, the all-position fit's
evaluations and its fwd/rev pair's evaluations when warm-started at the
all-position mode (MDFIT-MAP v1) or cold-started at the spec's initial point,
and the critical path each rule gives.

    python tools/pair_start_study.py [TAXA]
"""
import sys, numpy as np
sys.path.insert(0, '/root/repo')
from oracle.oracle import OracleLib as Oracle
from metadamage_amd.synthetic import generate
T = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
b = generate(T, seed=1)
o = Oracle()
rows = []
for t in range(T):
    y, N = b.y[t], b.N[t]
    for model in (0, 1):
        ua, Fa, ea, sa = o.fit_subfit(model, 0, y, N)
        warm = [o.fit_subfit(model, s, y, N, u0=ua if sa == 0 else None) for s in (1, 2)]
        cold = [o.fit_subfit(model, s, y, N) for s in (1, 2)]
        dF = max(abs(w[1] - c[1]) for w, c in zip(warm, cold))
        rows.append((t, model, ea, max(w[2] for w in warm), max(c[2] for c in cold), dF,
                     sum(w[3] != c[3] for w, c in zip(warm, cold))))
r = np.array(rows, float)
ea, pw, pc = r[:, 2], r[:, 3], r[:, 4]
cur = ea + pw
for K in (20, 30, 40):
    new = np.where(ea > K, np.maximum(ea, K + pc), ea + pw)
    print(f"K={K}: chain max cur {cur.max():.0f} new {new.max():.0f}; p99 cur {np.percentile(cur,99):.0f} new {np.percentile(new,99):.0f}; "
          f"p99.9 cur {np.percentile(cur,99.9):.0f} new {np.percentile(new,99.9):.0f}; taxa-models switched {(ea>K).mean()*100:.1f}%; "
          f"extra evals {((ea>K)*(pc-pw)).sum()/ (ea+pw).sum()*100:.2f}%")
print("max |F warm - F cold| over pairs:", r[:, 5].max(), " status diffs:", int(r[:, 6].sum()))
top = np.argsort(-cur)[:10]
for i in top: print("taxon", int(r[i,0]), "model", int(r[i,1]), "all", int(ea[i]), "pair warm", int(pw[i]), "pair cold", int(pc[i]))
