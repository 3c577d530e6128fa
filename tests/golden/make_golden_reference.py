"""Generate golden vectors from the reference's own Python code (run HERE only).

    python tests/golden/make_golden_reference.py

The reference (/root/reference/metadamage) cannot be imported as-is: jax,
numpyro, timeout_decorator, dask, PyPDF2, click_help_colors and toml are not
installed (ordinary ModuleNotFoundError).  Its jax-free
functions do run once those modules are replaced by empty stubs in
sys.modules.  This script does that and runs, from a
scratch cwd (metadamage/__init__.py creates ./logs):

  (1) the counts pipeline of counts.py:229-273 (dask steps restated as pandas:
      dd.read_csv -> the 20->22-column adapter below, dd.merge -> pd.merge,
      groupby.apply(meta=) -> groupby.apply) on the two shipped fixture
      files and on a seeded synthetic 22-column table, with the reference's
      add_reference_counts / add_error_rates / make_position_1_indexed /
      make_reverse_position_negative / replace_nans_with_zeroes /
      compute_y_sum_total / filter_cut_based_on_cfg / sort_by_alignments /
      downcast_dataframe;
  (2) group_to_numpyro_data (fits.py:398-419) and add_noise_estimates
      (fits.py:359-376) on every surviving taxon;
  (3) extract_top_max_fits (fits.py:736-744);
  (4) get_lppd_and_waic / compute_n_sigma /
      compute_assymmetry_combined_vs_forwardreverse (fits.py:147-227) on
      seeded log-likelihood matrices (S = 1 — the MAP case — and S = 50);
  (5) the record assembly compute_fit_results + add_assymetry_results_to_fit_results
      (fits.py:230-356) with MAP quantities injected at the numpyro boundary
      (fit_mcmc, compute_log_likelihood, get_y_average_and_hpdi,
      get_mean_of_variable are replaced by the MAP mode found by the scipy
      optimiser of make_golden_scipy.py), so the reference's own code decides
      column order, the 15/15 split and the D_max_reverse-on-data_forward quirk
      (the predictive HPDI comes from scipy's BetaBinomial pmf:
      make_golden_hpdi.hpdi_window, independent of the oracle and the kernel);
  (6) make_df_fit_results_from_fit_results / make_df_fit_predictions_from_d_fits
      column lists (fits.py:632-680).

Only data (inputs and expected outputs) is written to tests/golden/.
"""

from __future__ import annotations

import json
import os
import sys
import tempfile
import types
from pathlib import Path

import numpy as np
import pandas as pd

ROOT = Path(__file__).resolve().parents[2]
REF = Path("/root/reference")
OUT = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT))


def install_stubs():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    ident = lambda f=None, *a, **k: f  # noqa: E731
    jnp = mod("jax.numpy")
    jrandom = mod("jax.random", PRNGKey=lambda s: s)
    mod("jax", jit=ident, numpy=jnp, random=jrandom)
    dist = mod("numpyro.distributions")
    infer = mod("numpyro.infer", log_likelihood=None, MCMC=None, NUTS=None, Predictive=None)
    diag = mod("numpyro.diagnostics", hpdi=None)
    mod("numpyro", enable_x64=lambda: None, distributions=dist, infer=infer, diagnostics=diag,
        sample=None, deterministic=None)

    class _Timeout(Exception):
        pass

    mod("timeout_decorator", timeout=lambda t: (lambda f: f), TimeoutError=_Timeout)
    dd = mod("dask.dataframe")
    mod("dask.diagnostics", ProgressBar=object)
    mod("dask.distributed", Client=object, LocalCluster=object)
    mod("dask", dataframe=dd, delayed=ident)
    mod("PyPDF2", PdfFileReader=object)

    class _H:  # click_help_colors classes are only subclassed
        def __init__(self, *a, **k):
            pass

    mod("click_help_colors", HelpColorsCommand=_H, HelpColorsGroup=_H)
    mod("toml")


def read_fixture_20col(path: Path) -> pd.DataFrame:
    """Adapter: the shipped 20-column headed format
    (#taxid Nalignments Direction Pos AA..TT) -> the 22 columns counts.py:37-45
    expects.  tax_name / tax_rank are synthesised (the files carry none)."""
    raw = pd.read_csv(path, sep="\t")
    df = pd.DataFrame(
        {
            "tax_id": raw["#taxid"].astype(np.int64),
            "tax_name": raw["#taxid"].map(lambda t: f"taxid_{t}"),
            "tax_rank": "unknown",
            "N_alignments": raw["Nalignments"].astype(np.int64),
            "strand": raw["Direction"].astype(str),
            "position": raw["Pos"].astype(np.int64),
        }
    )
    for b in [r + o for r in "ACGT" for o in "ACGT"]:
        df[b] = raw[b].astype(np.int64)
    return df


def run_counts(counts, utils, df, cfg):
    """counts.compute_counts_with_dask (counts.py:212-273) with pandas."""
    fwd, rev = cfg.substitution_bases_forward, cfg.substitution_bases_reverse
    df = df.copy()
    df = counts.add_reference_counts(df, ref=fwd[0])
    df = counts.add_reference_counts(df, ref=rev[0])
    df = counts.add_error_rates(df, ref=fwd[0], obs=fwd[1])
    df = counts.add_error_rates(df, ref=rev[0], obs=rev[1])
    df = counts.make_position_1_indexed(df)
    df = counts.make_reverse_position_negative(df)
    df = counts.replace_nans_with_zeroes(df)
    ys = df.groupby("tax_id").apply(counts.compute_y_sum_total, cfg)
    ys = ys.rename("y_sum_total").reset_index()
    df = pd.merge(df, ys, on=["tax_id"])
    df = counts.filter_cut_based_on_cfg(df, cfg)
    df = df.reset_index(drop=True).pipe(counts.sort_by_alignments).reset_index(drop=True)
    df["shortname"] = cfg.shortname
    cats = ["tax_id", "tax_name", "tax_rank", "strand", "shortname"]
    return utils.downcast_dataframe(df, cats, fully_automatic=False)


class MapMCMC:
    """Stand-in for a numpyro MCMC object at the boundary the reference
    queries (fits.py:100,137,180,387): it 'fits' by looking up the MAP mode
    of (model, data subset) and exposes one posterior 'sample' = the mode."""

    def __init__(self, model, solver):
        self.sampler = types.SimpleNamespace(model=model)
        self.solver = solver
        self.data = None
        self.theta = None

    def run(self, data):
        self.data = {k: np.asarray(v) for k, v in data.items()}
        self.theta = self.solver(self.sampler.model.__name__, self.data)

    def get_samples(self):
        q, A, c, phi = self.theta
        D_max = A + c if self.sampler.model.__name__ == "model_PMD" else q
        return {"q": np.array([q]), "phi": np.array([phi]), "D_max": np.array([D_max])}


def main():
    install_stubs()
    sys.path.insert(0, str(REF))
    scratch = tempfile.mkdtemp(prefix="mdgold_")
    cwd = os.getcwd()
    os.chdir(scratch)
    try:
        from metadamage import counts, fits, utils  # noqa: E402
    finally:
        os.chdir(cwd)

    from scipy import special

    import make_golden_scipy as msc  # restated objective + optimiser (no reference code)
    from metadamage_amd.synthetic import generate, to_counts_table

    res: dict[str, np.ndarray] = {}
    meta: dict = {"cases": {}}

    def make_cfg(name, min_alignments=10, min_y_sum=10, fwd="CT", rev="GA", max_fits=None):
        cfg = utils.Config(out_dir=Path(scratch) / "out", max_fits=max_fits, max_cores=1,
                           min_alignments=min_alignments, min_y_sum=min_y_sum,
                           substitution_bases_forward=fwd, substitution_bases_reverse=rev,
                           forced=False, version="0.0.0")
        cfg.add_filename(f"{name}.txt")
        return cfg

    # ---------------- (1)-(3) counts, packing, noise, top-N -----------------
    synth = to_counts_table(generate(40, seed=5, fail_fraction=0.3))
    synth_path = OUT / "synthetic_counts_22col.tsv"
    synth.to_csv(synth_path, sep="\t", header=False, index=False)
    cases = [
        ("data_ancient", read_fixture_20col(REF / "data/input/data_ancient.txt"), {}),
        ("data_control", read_fixture_20col(REF / "data/input/data_control.txt"), {}),
        ("synthetic", pd.read_csv(synth_path, sep="\t", header=None, names=counts.columns), {}),
        ("synthetic_strict", pd.read_csv(synth_path, sep="\t", header=None, names=counts.columns),
         dict(min_alignments=20000, min_y_sum=2000)),
        ("synthetic_CA_GT", pd.read_csv(synth_path, sep="\t", header=None, names=counts.columns),
         dict(fwd="CA", rev="GT")),
    ]
    for name, raw, kw in cases:
        cfg = make_cfg(name, **kw)
        df = run_counts(counts, utils, raw, cfg)
        df.to_parquet(OUT / f"counts_{name}.parquet")
        groups = list(df.groupby("tax_id", sort=False, observed=True))
        ys, Ns, zs, noise, tids = [], [], [], [], []
        for tax_id, group in groups:
            d = fits.group_to_numpyro_data(group, cfg)
            fr = {}
            fits.add_noise_estimates(group, fr)
            ys.append(d["y"]); Ns.append(d["N"]); zs.append(d["z"]); tids.append(int(tax_id))
            noise.append([fr["normalized_noise"], fr["normalized_noise_forward"], fr["normalized_noise_reverse"]])
        T = len(groups)
        res[f"{name}__tax_id"] = np.array(tids, dtype=np.int64)
        res[f"{name}__y"] = np.array(ys, dtype=np.int64).reshape(T, 30)
        res[f"{name}__N"] = np.array(Ns, dtype=np.int64).reshape(T, 30)
        res[f"{name}__z"] = np.array(zs, dtype=np.int64).reshape(T, 30)
        res[f"{name}__noise"] = np.array(noise, dtype=float).reshape(T, 3)
        tops = {}
        for k in (1, 2, 5, 100):
            tops[str(k)] = [int(t) for t in pd.unique(fits.get_top_max_fits(df, k).tax_id)]
        meta["cases"][name] = {"cfg": {k: (str(v) if isinstance(v, Path) else v)
                                       for k, v in cfg.to_dict().items()},
                               "n_taxa": T, "top_max_fits": tops, "columns": list(df.columns)}
        print(name, "taxa after cuts:", T)

    # ---------------- (4) WAIC / n_sigma / asymmetry --------------------------
    rng = np.random.default_rng(2024)
    orig_cll = fits.compute_log_likelihood
    fits.compute_log_likelihood = lambda mat, data: mat  # the matrix IS the 'mcmc'
    waic_cases = []
    for S in (1, 50, 50):
        lP = rng.normal(-5, 2, (S, 30)) - rng.uniform(0, 3, 30)
        lN = lP - rng.uniform(0, 4, 30) + rng.normal(0, 0.3, (S, 30))
        lF = lP[:, :15] + rng.normal(0, 0.5, (S, 15))
        lR = lP[:, 15:] + rng.normal(0, 0.5, (S, 15))
        lNF = lF - rng.uniform(0, 2, 15)
        dP, dN = fits.get_lppd_and_waic(lP, None), fits.get_lppd_and_waic(lN, None)
        dF, dR = fits.get_lppd_and_waic(lF, None), fits.get_lppd_and_waic(lR, None)
        dNF = fits.get_lppd_and_waic(lNF, None)
        waic_cases.append(dict(
            lP=lP, lN=lN, lF=lF, lR=lR, lNF=lNF,
            waic_i_P=dP["waic_i"], waic_P=dP["waic"], lppd_P=dP["lppd"], pWAIC_P=dP["pWAIC"],
            n_sigma=fits.compute_n_sigma(dP, dN), n_sigma_fwd=fits.compute_n_sigma(dF, dNF),
            asymmetry=fits.compute_assymmetry_combined_vs_forwardreverse(dP, dF, dR)))
    fits.compute_log_likelihood = orig_cll
    for i, c in enumerate(waic_cases):
        for k, v in c.items():
            res[f"waic{i}__{k}"] = np.asarray(v, dtype=float)
    meta["n_waic_cases"] = len(waic_cases)

    # ---------------- (5) record assembly with MAP quantities ------------------
    def theta_of(u, model_name):
        q = special.expit(u[0])
        phi = np.exp(u[3]) + 2.0
        if model_name == "model_PMD":
            return (q, special.expit(u[1]), u[2], phi)
        return (q, 0.0, 0.0, phi)

    def solver(model_name, data):
        z = data["z"]
        lo, hi = (0, 30) if len(z) == 30 else ((0, 15) if z[0] > 0 else (15, 30))
        y30 = np.zeros(30, np.uint32); N30 = np.zeros(30, np.uint32)
        y30[lo:hi] = data["y"]; N30[lo:hi] = data["N"]
        model = 0 if model_name == "model_PMD" else 1
        F, u = msc.map_fit(model, y30, N30, lo, hi, msc.starts_for(model))
        return theta_of(u, model_name)

    def pointwise_ell(theta, data, pmd):
        q, A, c, phi = theta
        y = data["y"].astype(float); N = data["N"].astype(float)
        k = np.abs(data["z"]) - 1.0
        D = np.clip(A * (1 - q) ** k + c, 0, 1) if pmd else np.full_like(y, q)
        a, b = D * phi, (1 - D) * phi
        return (special.gammaln(N + 1) - special.gammaln(y + 1) - special.gammaln(N - y + 1)
                + special.gammaln(y + a) + special.gammaln(N - y + b) - special.gammaln(N + phi)
                - special.gammaln(a) - special.gammaln(b) + special.gammaln(phi))

    import make_golden_hpdi as mgh  # scipy's shortest 68 % window of the predictive BetaBinomial

    def map_predictive(mcmc, data, func=np.median, return_hpdi=True):
        """get_y_average_and_hpdi (fits.py:112-120) with the mode as the one
        posterior sample: median := D(z); HPDI := the shortest window of
        BetaBinomial(D phi, (1-D) phi, N) / N holding 68 % (scipy pmf)."""
        q, A, c, phi = mcmc.theta
        N = data["N"].astype(float)
        k = np.abs(data["z"]) - 1.0
        D = np.minimum(A * (1 - q) ** k + c, 1.0)
        med = np.where(N > 0, D, np.nan)
        if not return_hpdi:
            return med
        lo = np.full_like(N, np.nan)
        hi = np.full_like(N, np.nan)
        for i in range(N.size):
            if N[i] > 0:
                wl, wh = mgh.hpdi_window(N[i], D[i] * phi, (1 - D[i]) * phi)
                lo[i], hi[i] = wl / N[i], wh / N[i]
        return med, np.stack([lo, hi])

    fits.fit_mcmc = lambda mcmc, data, seed=0: mcmc.run(data)
    fits.compute_log_likelihood = lambda mcmc, data: pointwise_ell(
        mcmc.theta, data, mcmc.sampler.model.__name__ == "model_PMD")[None, :]
    fits.get_y_average_and_hpdi = map_predictive
    for name in ("data_ancient", "data_control", "synthetic"):
        cfg = make_cfg(name)
        df = pd.read_parquet(OUT / f"counts_{name}.parquet")
        df["tax_id"] = df["tax_id"].astype("category")
        records, medians, hpdis, keys = [], [], [], None
        for i, (tax_id, group) in enumerate(df.groupby("tax_id", sort=False, observed=True)):
            if name == "synthetic" and i >= 12:
                break
            mP, mN = MapMCMC(fits.model_PMD, solver), MapMCMC(fits.model_null, solver)
            mPfr, mNfr = MapMCMC(fits.model_PMD, solver), MapMCMC(fits.model_null, solver)
            d_fit = fits.fit_single_group_without_timeout(group, cfg, mP, mN, mPfr, mNfr)
            fr = d_fit["fit_result"]
            keys = list(fr.keys())
            records.append([float(fr[k]) for k in keys[3:]])
            medians.append(np.asarray(d_fit["median"], float))
            hpdis.append(np.asarray(d_fit["hpdi"], float))
        res[f"record_{name}__values"] = np.array(records)
        res[f"record_{name}__median"] = np.array(medians)
        res[f"record_{name}__hpdi"] = np.array(hpdis)
        meta["record_keys"] = keys
        # (6) frame builders -> column lists
        d_fits = {}
        for tax_id, (rec, med, hp) in zip(res[f"{name}__tax_id"], zip(records, medians, hpdis)):
            fr = dict(zip(keys, [tax_id, f"taxid_{tax_id}", "unknown"] + list(rec)))
            d_fits[tax_id] = {"fit_result": fr, "median": med, "hpdi": hp}
        fit_results = {t: d["fit_result"] for t, d in d_fits.items()}
        dfr = fits.make_df_fit_results_from_fit_results(fit_results, df, cfg)
        dfp = fits.make_df_fit_predictions_from_d_fits(d_fits, cfg)
        meta["fit_results_columns"] = list(dfr.columns)
        meta["fit_predictions_columns"] = list(dfp.columns)
        meta["fit_predictions_position"] = [int(p) for p in dfp["position"][:30]]
        print("record", name, len(records))

    np.savez_compressed(OUT / "reference_golden.npz", **res)
    (OUT / "reference_golden.json").write_text(json.dumps(meta, indent=1, default=str))
    print("wrote tests/golden/reference_golden.{npz,json}")


if __name__ == "__main__":
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    main()
