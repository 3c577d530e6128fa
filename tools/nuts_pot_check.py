"""GPU sampling-mode potential vs the oracle's (development check)."""
import sys
from pathlib import Path
import numpy as np
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from metadamage_amd import engine
from metadamage_amd.synthetic import generate
from oracle.oracle import OracleLib

b = generate(40, seed=3)
o = OracleLib()
rng = np.random.default_rng(0)
items = [(t, m, s) for t in range(40) for m in (0, 1) for s in (0, 1, 2)]
model = np.array([m for _, m, _ in items]); subset = np.array([s for _, _, s in items])
y = b.y[[t for t, _, _ in items]]; N = b.N[[t for t, _, _ in items]]
v = rng.uniform(-2, 2, (len(items), 4)); v[model == 1, 1:3] = 0
U, g = engine.nuts_potential(model, subset, y, N, v)
worst = 0
for k, (t, m, s) in enumerate(items):
    Uo, go = o.nuts_potential(m, s, y[k, :30], N[k, :30], v[k])
    if not np.isfinite(Uo) or not np.isfinite(U[k]):
        if np.isfinite(Uo) != np.isfinite(U[k]):
            print("finiteness mismatch", t, m, s, U[k], Uo)
        continue
    eU = abs(U[k] - Uo) / max(1, abs(Uo)); eg = np.abs(g[k] - go).max() / max(1, np.abs(go).max())
    worst = max(worst, eU, eg)
    if eU > 1e-12 or eg > 1e-9:
        print(t, m, s, "U", U[k], Uo, "g", g[k], go)
print("worst", worst)
