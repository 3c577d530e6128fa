// counts.cpp — the count pipeline of the reference's ingest on parsed rows
// (include/mdingest.h: mdi_select / mdi_gather).
//
// Restates /root/reference/metadamage/counts.py:86-209 for the columns
// mdi_parse_into produced:
//   add_reference_counts   counts.py:86-89    ref = sum of the 4 pairs starting with the base
//   add_error_rates        counts.py:109-114  f = count / ref (0/0 -> 0, x/0 -> inf)
//   positions              counts.py:117-126  1-indexed, reverse strand negative
//   y_sum_total            counts.py:179-204  per tax_id sum of the substitution counts
//   cut                    counts.py:207-209  N_alignments >= min_alignments & y_sum_total >= min_y_sum
//   sort_by_alignments     counts.py:167-172  N_alignments, tax_id, 1/z | z, all descending
//   downcast               utils.py:329-356   ints -> uint32 (position int8), floats -> float32
// The vectorised numpy restatement of the same steps (metadamage_amd/ingest.py
// history, counts.compute_counts_pandas line by line) is the parity check.
//
// mdi_select finds the kept rows and their order (one pass, plus a sort of
// the taxa in the usual layout: each tax_id's rows contiguous and already in
// z order); mdi_gather writes the output columns of the kept rows in that
// order, one row range per thread.

#include <stdint.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/mdingest.h"

namespace {

struct Rows {
  int64_t n;
  const int64_t* tax_id;
  const int64_t* nal;
  const int64_t* position;
  const int64_t* counts;  // [16][n]
  const int32_t* strand_code;
  const uint8_t* code_is_fwd;
  int n_codes;
  const int64_t* col(int k) const { return counts + (int64_t)k * n; }
  bool fwd(int64_t r) const {
    const int32_t c = strand_code[r];
    return c >= 0 && c < n_codes && code_is_fwd[c];
  }
  int64_t pos(int64_t r) const { return fwd(r) ? position[r] + 1 : -(position[r] + 1); }
};

// "AC" -> column index in AA AC .. TT order; -1 if not a base pair
int pair_index(const char* s) {
  static const char kBases[] = "ACGT";
  if (!s || std::strlen(s) != 2) return -1;
  const char* a = std::strchr(kBases, s[0]);
  const char* b = std::strchr(kBases, s[1]);
  if (!a || !b || !s[0] || !s[1]) return -1;
  return (int)(a - kBases) * 4 + (int)(b - kBases);
}

double order_key(int64_t p) { return p > 0 ? 1.0 / (double)p : (double)p; }

thread_local char g_cerr[256] = "";

int pool_size(int n_threads, int64_t n) {
  int nt = n_threads > 0 ? n_threads : mdi_default_threads();
  if (nt < 1) nt = 1;
  if (n < (int64_t)nt * 65536) nt = (int)std::max<int64_t>(1, n / 65536);
  return nt > 64 ? 64 : nt;
}

template <typename F>
void for_ranges(int nt, int64_t n, F f) {
  if (nt <= 1) {
    f(0, (int64_t)0, n);
    return;
  }
  std::vector<std::thread> pool;
  for (int i = 0; i < nt; ++i) pool.emplace_back(f, i, n * i / nt, n * (i + 1) / nt);
  for (auto& t : pool) t.join();
}


int arg_error(const char* what) {
  std::snprintf(g_cerr, sizeof g_cerr, "%s", what);
  return MDI_E_ARG;
}

}  // namespace

extern "C" {

int64_t mdi_select(int64_t rows, const int64_t* tax_id, const int64_t* n_alignments, const int64_t* position,
                   const int64_t* counts16, const int32_t* strand_code, const uint8_t* code_is_fwd,
                   int32_t n_codes, const char* sub_fwd, const char* sub_rev, int64_t min_alignments,
                   int64_t min_y_sum, int n_threads, int32_t* taxon, int64_t* y_sum_total, int64_t* perm,
                   int64_t* uniq, int64_t* n_taxa) {
  if (rows < 0 || (rows > 0 && (!tax_id || !n_alignments || !position || !counts16 || !strand_code ||
                                !taxon || !y_sum_total || !perm)) ||
      n_codes < 0 || (n_codes > 0 && !code_is_fwd))
    return arg_error("mdi_select: bad arguments");
  const int kf = pair_index(sub_fwd), kr = pair_index(sub_rev);
  if (kf < 0 || kr < 0) return arg_error("mdi_select: substitutions must be base pairs like \"CT\"");
  const Rows R{rows, tax_id, n_alignments, position, counts16, strand_code, code_is_fwd, n_codes};
  const int64_t* yf = R.col(kf);
  const int64_t* yr = R.col(kr);
  const int nt = pool_size(n_threads, rows);

  // (1) per row range: the runs of equal tax_id and their substitution sums
  struct Run {
    int64_t start, tax, ys;
  };
  std::vector<std::vector<Run>> runs((size_t)nt);
  for_ranges(nt, rows, [&](int tid, int64_t lo, int64_t hi) {
    std::vector<Run>& v = runs[(size_t)tid];
    for (int64_t r = lo; r < hi; ++r) {
      if (r == lo || tax_id[r] != tax_id[r - 1]) v.push_back({r, tax_id[r], 0});
      const int64_t p = R.pos(r);
      v.back().ys += p > 0 ? yf[r] : (p < 0 ? yr[r] : 0);
    }
  });
  // (2) taxon index in first-appearance order (pd.factorize) over the runs, in file order
  std::unordered_map<int64_t, int32_t> index;
  std::vector<int64_t> ysum, utax;
  std::vector<std::vector<int32_t>> run_id((size_t)nt);
  for (int tid = 0; tid < nt; ++tid)
    for (const Run& u : runs[(size_t)tid]) {
      auto it = index.emplace(u.tax, (int32_t)ysum.size());
      if (it.second) {
        ysum.push_back(0);
        utax.push_back(u.tax);
      }
      ysum[(size_t)it.first->second] += u.ys;
      run_id[(size_t)tid].push_back(it.first->second);
    }
  // (3) per row: its taxon and y_sum_total, the cut; (4) the kept rows in file order
  std::vector<int64_t> kept((size_t)nt + 1, 0);
  for_ranges(nt, rows, [&](int tid, int64_t lo, int64_t hi) {
    const std::vector<Run>& v = runs[(size_t)tid];
    int64_t k = 0;
    for (size_t j = 0; j < v.size(); ++j) {
      const int32_t id = run_id[(size_t)tid][j];
      const int64_t ys = ysum[(size_t)id];
      const int64_t e = j + 1 < v.size() ? v[j + 1].start : hi;
      for (int64_t r = v[j].start; r < e; ++r) {
        taxon[r] = id;
        y_sum_total[r] = ys;
        k += n_alignments[r] >= min_alignments && ys >= min_y_sum;
      }
    }
    kept[(size_t)tid + 1] = k;
  });
  for (int tid = 0; tid < nt; ++tid) kept[(size_t)tid + 1] += kept[(size_t)tid];
  const int64_t n_keep = kept[(size_t)nt];
  for_ranges(nt, rows, [&](int tid, int64_t lo, int64_t hi) {
    int64_t w = kept[(size_t)tid];
    for (int64_t r = lo; r < hi; ++r)
      if (n_alignments[r] >= min_alignments && y_sum_total[r] >= min_y_sum) perm[w++] = r;
  });
  if (n_taxa) *n_taxa = (int64_t)utax.size();
  if (uniq && !utax.empty()) std::memcpy(uniq, utax.data(), sizeof(int64_t) * utax.size());

  // sort_by_alignments.  Usual layout: every taxon's kept rows one contiguous
  // run, z order already descending within it, one N_alignments per run ->
  // sort the runs only.  Otherwise the full three-key sort (stable: ties keep
  // file order, as np.lexsort).
  const int kt = pool_size(n_threads, n_keep);
  std::vector<std::vector<int64_t>> tstarts((size_t)kt);
  std::vector<uint8_t> tok((size_t)kt, 1);
  for_ranges(kt, n_keep, [&](int tid, int64_t lo, int64_t hi) {
    std::vector<int64_t>& st = tstarts[(size_t)tid];
    for (int64_t i = lo; i < hi; ++i) {
      const int64_t r = perm[i];
      if (i == 0 || taxon[r] != taxon[perm[i - 1]]) {
        st.push_back(i);
      } else {
        const int64_t q = perm[i - 1];
        if (!(order_key(R.pos(r)) < order_key(R.pos(q))) || n_alignments[r] != n_alignments[q]) {
          tok[(size_t)tid] = 0;
          return;
        }
      }
    }
  });
  bool runs_ok = true;
  for (int tid = 0; tid < kt; ++tid) runs_ok = runs_ok && tok[(size_t)tid];
  std::vector<int64_t> starts;
  if (runs_ok) {
    std::vector<uint8_t> seen(ysum.size(), 0);
    for (int tid = 0; tid < kt && runs_ok; ++tid)
      for (const int64_t i : tstarts[(size_t)tid]) {
        const int32_t t = taxon[perm[i]];
        if (seen[(size_t)t]) {
          runs_ok = false;
          break;
        }
        seen[(size_t)t] = 1;
        starts.push_back(i);
      }
  }
  if (runs_ok) {
    const size_t nb = starts.size();
    struct Key {
      int64_t nal, tax, b;
    };
    std::vector<Key> keys(nb);
    for (size_t b = 0; b < nb; ++b) {
      const int64_t r = perm[starts[b]];
      keys[b] = {n_alignments[r], tax_id[r], (int64_t)b};
    }
    std::sort(keys.begin(), keys.end(), [](const Key& a, const Key& b) {
      if (a.nal != b.nal) return a.nal > b.nal;
      if (a.tax != b.tax) return a.tax > b.tax;
      return a.b < b.b;
    });
    std::vector<int64_t> dst(nb + 1, 0);
    for (size_t k = 0; k < nb; ++k) {
      const int64_t b = keys[k].b;
      const int64_t hi = (size_t)b + 1 < nb ? starts[(size_t)b + 1] : n_keep;
      dst[k + 1] = dst[k] + (hi - starts[(size_t)b]);
    }
    std::vector<int64_t> out((size_t)n_keep);
    for_ranges(pool_size(n_threads, (int64_t)nb * 32), (int64_t)nb, [&](int, int64_t lo, int64_t hi) {
      for (int64_t k = lo; k < hi; ++k) {
        const int64_t b = keys[(size_t)k].b;
        std::memcpy(out.data() + dst[(size_t)k], perm + starts[(size_t)b],
                    sizeof(int64_t) * (size_t)(dst[(size_t)k + 1] - dst[(size_t)k]));
      }
    });
    if (n_keep > 0) std::memcpy(perm, out.data(), sizeof(int64_t) * (size_t)n_keep);
  } else {
    std::stable_sort(perm, perm + n_keep, [&](int64_t a, int64_t b) {
      if (n_alignments[a] != n_alignments[b]) return n_alignments[a] > n_alignments[b];
      if (tax_id[a] != tax_id[b]) return tax_id[a] > tax_id[b];
      return order_key(R.pos(a)) > order_key(R.pos(b));
    });
  }
  return n_keep;
}

int mdi_gather(int64_t rows, const int64_t* perm, int64_t n_keep, const int64_t* n_alignments,
               const int64_t* position, const int64_t* counts16, const int32_t* strand_code,
               const uint8_t* code_is_fwd, int32_t n_codes, const char* sub_fwd, const char* sub_rev,
               const int64_t* y_sum_total, int n_threads, uint32_t* o_nal, int8_t* o_position,
               uint32_t* o_counts16, uint32_t* o_ref2, float* o_f2, uint32_t* o_y_sum_total) {
  if (n_keep < 0 || (n_keep > 0 && (!perm || !n_alignments || !position || !counts16 || !strand_code ||
                                    !y_sum_total || !o_nal || !o_position || !o_counts16 || !o_ref2 ||
                                    !o_f2 || !o_y_sum_total)))
    return arg_error("mdi_gather: bad arguments");
  const int kf = pair_index(sub_fwd), kr = pair_index(sub_rev);
  if (kf < 0 || kr < 0) return arg_error("mdi_gather: substitutions must be base pairs like \"CT\"");
  const Rows R{rows, nullptr, n_alignments, position, counts16, strand_code, code_is_fwd, n_codes};
  const int ref_base[2] = {kf / 4, kr / 4};
  const int sub[2] = {kf, kr};
  int nt = n_threads > 0 ? n_threads : mdi_default_threads();
  if (nt < 1) nt = 1;
  if (n_keep < (int64_t)nt * 65536) nt = (int)std::max<int64_t>(1, n_keep / 65536);
  if (nt > 64) nt = 64;
  std::vector<uint8_t> overflow((size_t)nt, 0);  // per thread: a kept value above uint32 (utils.py:338-339)
  auto work = [&](int tid, int64_t lo, int64_t hi) {
    const int64_t big = 0xFFFFFFFFll;
    bool ovf = false;
    for (int64_t i = lo; i < hi; ++i) {
      const int64_t r = perm[i];
      const int64_t nal = n_alignments[r];
      ovf |= nal > big;
      o_nal[i] = (uint32_t)nal;
      o_position[i] = (int8_t)R.pos(r);
      for (int k = 0; k < 16; ++k) {
        const int64_t v = R.col(k)[r];
        ovf |= v > big;
        o_counts16[(int64_t)k * n_keep + i] = (uint32_t)v;
      }
      for (int s = 0; s < 2; ++s) {
        const int b = ref_base[s];
        const int64_t ref = R.col(4 * b)[r] + R.col(4 * b + 1)[r] + R.col(4 * b + 2)[r] + R.col(4 * b + 3)[r];
        ovf |= ref > big;
        o_ref2[(int64_t)s * n_keep + i] = (uint32_t)ref;
        const int64_t c = R.col(sub[s])[r];
        double f;
        if (ref != 0) f = (double)c / (double)ref;
        else f = c == 0 ? 0.0 : (c > 0 ? __builtin_inf() : -__builtin_inf());
        o_f2[(int64_t)s * n_keep + i] = (float)f;
      }
      const int64_t ys = y_sum_total[r];
      ovf |= ys > big;
      o_y_sum_total[i] = (uint32_t)ys;
    }
    overflow[tid] = ovf;
  };
  if (nt == 1) {
    work(0, 0, n_keep);
  } else {
    std::vector<std::thread> pool;
    for (int i = 0; i < nt; ++i) pool.emplace_back(work, i, n_keep * i / nt, n_keep * (i + 1) / nt);
    for (auto& t : pool) t.join();
  }
  for (int i = 0; i < nt; ++i)
    if (overflow[i]) {
      std::snprintf(g_cerr, sizeof g_cerr, "Dataframe contains too large values.");
      return MDI_E_RANGE;
    }
  return 0;
}

const char* mdi_counts_error(void) { return g_cerr; }

}  // extern "C"

extern "C" {

int mdi_codes(int64_t n_keep, const int64_t* perm, int n_cols, const int32_t* const* in, const int32_t* n_table,
              int n_threads, int32_t* const* out, uint8_t* const* used) {
  if (n_keep < 0 || n_cols < 0 || n_cols > 8 || (n_cols > 0 && (!in || !n_table || !out || !used)) ||
      (n_keep > 0 && !perm))
    return arg_error("mdi_codes: bad arguments");
  for (int c = 0; c < n_cols; ++c) {
    if (n_table[c] < 0 || !in[c] || !out[c] || !used[c]) return arg_error("mdi_codes: bad column");
    std::memset(used[c], 0, (size_t)n_table[c]);
  }
  const int nt = pool_size(n_threads, n_keep);
  // per-thread usage flags, OR-merged (the tables are per taxon at most: small)
  std::vector<std::vector<uint8_t>> seen((size_t)nt * (size_t)n_cols);
  std::vector<uint8_t> bad((size_t)nt, 0);
  for_ranges(nt, n_keep, [&](int tid, int64_t lo, int64_t hi) {
    for (int c = 0; c < n_cols; ++c) {
      std::vector<uint8_t>& u = seen[(size_t)tid * n_cols + c];
      u.assign((size_t)n_table[c], 0);
      const int32_t* src = in[c];
      int32_t* dst = out[c];
      const int32_t m = n_table[c];
      for (int64_t i = lo; i < hi; ++i) {
        const int32_t k = src[perm[i]];
        if (k < 0 || k >= m) {
          bad[tid] = 1;
          continue;
        }
        dst[i] = k;
        u[(size_t)k] = 1;
      }
    }
  });
  for (int i = 0; i < nt; ++i)
    if (bad[i]) return arg_error("mdi_codes: code out of its table");
  for (int c = 0; c < n_cols; ++c)
    for (int i = 0; i < nt; ++i) {
      const std::vector<uint8_t>& u = seen[(size_t)i * n_cols + c];
      for (size_t k = 0; k < u.size(); ++k) used[c][k] |= u[k];
    }
  return 0;
}

int mdi_remap(int64_t n, int n_cols, int32_t* const* codes, const int32_t* const* remap, int n_threads) {
  if (n < 0 || n_cols < 0 || (n_cols > 0 && (!codes || !remap))) return arg_error("mdi_remap: bad arguments");
  for (int c = 0; c < n_cols; ++c)
    if (!codes[c] || !remap[c]) return arg_error("mdi_remap: bad column");
  for_ranges(pool_size(n_threads, n), n, [&](int, int64_t lo, int64_t hi) {
    for (int c = 0; c < n_cols; ++c) {
      int32_t* x = codes[c];
      const int32_t* m = remap[c];
      for (int64_t i = lo; i < hi; ++i) x[i] = m[x[i]];
    }
  });
  return 0;
}

int64_t mdi_first_index(int64_t n, const int32_t* codes, int32_t n_cat, int64_t* taxon, int64_t* first) {
  if (n < 0 || n_cat < 0 || (n > 0 && (!codes || !taxon || !first))) return arg_error("mdi_first_index: bad arguments");
  std::vector<int64_t> index((size_t)n_cat, -1);
  int64_t T = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int32_t k = codes[i];
    if (k < 0 || k >= n_cat) return arg_error("mdi_first_index: code out of its table");
    int64_t& t = index[(size_t)k];
    if (t < 0) {
      t = T;
      first[T++] = i;
    }
    taxon[i] = t;
  }
  return T;
}

int mdi_interleave(int64_t n, int n_cols, const uint32_t* const* cols, uint32_t* out, int n_threads) {
  if (n < 0 || n_cols < 1 || n_cols > 64 || (n > 0 && (!cols || !out))) return arg_error("mdi_interleave: bad arguments");
  for (int c = 0; c < n_cols; ++c)
    if (n > 0 && !cols[c]) return arg_error("mdi_interleave: bad column");
  // row blocks of 2048: the block's slices of every column stay in L1/L2
  // while the interleaved rows are written out sequentially
  for_ranges(pool_size(n_threads, n), n, [&](int, int64_t lo, int64_t hi) {
    for (int64_t a = lo; a < hi; a += 2048) {
      const int64_t b = std::min<int64_t>(hi, a + 2048);
      for (int c = 0; c < n_cols; ++c) {
        const uint32_t* src = cols[c];
        uint32_t* dst = out + c;
        for (int64_t i = a; i < b; ++i) dst[i * n_cols] = src[i];
      }
    }
  });
  return 0;
}

int64_t mdi_used_codes(int64_t n, const int32_t* codes, int32_t n_cat, int n_threads, uint8_t* used,
                       int64_t* n_missing) {
  if (n < 0 || n_cat < 0 || (n > 0 && !codes) || (n_cat > 0 && !used)) return arg_error("mdi_used_codes: bad arguments");
  const int nt = pool_size(n_threads, n);
  std::vector<std::vector<uint8_t>> seen((size_t)nt);
  std::vector<int64_t> miss((size_t)nt, 0);
  std::vector<uint8_t> bad((size_t)nt, 0);
  for_ranges(nt, n, [&](int tid, int64_t lo, int64_t hi) {
    std::vector<uint8_t>& u = seen[(size_t)tid];
    u.assign((size_t)n_cat, 0);
    int64_t m = 0;
    bool b = false;
    for (int64_t i = lo; i < hi; ++i) {
      const int32_t k = codes[i];
      if (k < 0) {
        ++m;
      } else if (k >= n_cat) {
        b = true;
      } else {
        u[(size_t)k] = 1;
      }
    }
    miss[(size_t)tid] = m;
    bad[(size_t)tid] = b;
  });
  int64_t m = 0;
  for (int i = 0; i < nt; ++i) {
    if (bad[(size_t)i]) return arg_error("mdi_used_codes: code out of its table");
    m += miss[(size_t)i];
  }
  if (n_missing) *n_missing = m;
  std::vector<int64_t> cnt((size_t)nt, 0);
  for_ranges(pool_size(n_threads, n_cat), n_cat, [&](int tid, int64_t lo, int64_t hi) {
    int64_t c = 0;
    for (int64_t k = lo; k < hi; ++k) {
      uint8_t v = 0;
      for (int i = 0; i < nt; ++i) v |= seen[(size_t)i][(size_t)k];
      used[k] = v;
      c += v;
    }
    cnt[(size_t)tid] = c;
  });
  int64_t k = 0;
  for (int64_t c : cnt) k += c;
  return k;
}

int64_t mdi_pack_dense(int64_t n, const int32_t* codes, int32_t n_cat, const int8_t* position,
                       const uint32_t* const* cols, int ld, int n_threads, uint32_t* y, uint32_t* N, uint32_t* mm) {
  constexpr int kPos = 30, kMM = 12;
  if (n < 0 || n_cat < 0 || ld < kPos || (n > 0 && (!codes || !position || !cols || !y || !N || !mm)))
    return arg_error("mdi_pack_dense: bad arguments");
  for (int c = 0; c < kMM + 4; ++c)
    if (n > 0 && !cols[c]) return arg_error("mdi_pack_dense: bad column");
  if (n % kPos) return MDI_E_LAYOUT;
  const int64_t T = n / kPos;
  // one pass over the blocks: write them, and check the layout on the way
  // (a failed check returns MDI_E_LAYOUT; the caller's general path rewrites everything)
  const int nt = pool_size(n_threads, n);
  std::vector<uint8_t> bad((size_t)nt, 0);
  for_ranges(nt, T, [&](int tid, int64_t lo, int64_t hi) {
    bool b = false;
    for (int64_t t = lo; t < hi; ++t) {
      const int64_t r0 = t * kPos;
      const int32_t k = codes[r0];
      b |= k < 0 || k >= n_cat;
      uint32_t* yt = y + t * ld;
      uint32_t* Nt = N + t * ld;
      for (int j = 0; j < kPos; ++j) {
        const int64_t r = r0 + j;
        const int want = j < 15 ? j + 1 : 14 - j;  // z = 1..15, -1..-15
        b |= codes[r] != k || position[r] != want;
        const int s = j < 15 ? 0 : 1;
        yt[j] = cols[kMM + s][r];
        Nt[j] = cols[kMM + 2 + s][r];
        uint32_t* m = mm + r * kMM;
        for (int c = 0; c < kMM; ++c) m[c] = cols[c][r];
      }
      for (int j = kPos; j < ld; ++j) yt[j] = Nt[j] = 0;
    }
    bad[(size_t)tid] = b;
  });
  for (int i = 0; i < nt; ++i)
    if (bad[(size_t)i]) return MDI_E_LAYOUT;
  // no tax_id code in two blocks (each taxon's rows contiguous)
  std::vector<uint8_t> seen((size_t)n_cat, 0);
  for (int64_t t = 0; t < T; ++t) {
    uint8_t& s = seen[(size_t)codes[t * kPos]];
    if (s) return MDI_E_LAYOUT;
    s = 1;
  }
  return T;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// mdi_noise: fits.py:359-376 per packed taxon (the oracle's noise() is the check)
// ---------------------------------------------------------------------------
namespace {
constexpr int kNPos = 30, kNHalf = 15, kNMM = 12, kCT = 5, kGA = 6;

void noise_one(const uint32_t* mm, double* out3) {
  // per column: 1 / mean over its valid rows (CT forward, GA reverse excluded);
  // a column of zeros has mean 0 -> every X = 0/0 = NaN -> dropped (np.nanstd).
  // Branch-free over the fixed 30 x 12 block: a 0/1 weight per entry.
  double inv[kNMM], okc[kNMM];
  for (int j = 0; j < kNMM; ++j) {
    uint64_t s = 0;
    for (int i = 0; i < kNPos; ++i) {
      const bool ex = (j == kCT && i < kNHalf) || (j == kGA && i >= kNHalf);
      s += ex ? 0u : mm[i * kNMM + j];
    }
    const int cnt = (j == kCT || j == kGA) ? kNHalf : kNPos;
    okc[j] = s != 0 ? 1.0 : 0.0;
    inv[j] = s != 0 ? (double)cnt / (double)s : 0.0;
  }
  double x[kNPos][kNMM], w[kNPos][kNMM];
  double sum[2] = {0.0, 0.0}, cnt[2] = {0.0, 0.0};
  for (int i = 0; i < kNPos; ++i) {
    const int h = i >= kNHalf;
    double sh = 0.0, ch = 0.0;
    for (int j = 0; j < kNMM; ++j) {
      const double ex = ((j == kCT && i < kNHalf) || (j == kGA && i >= kNHalf)) ? 0.0 : 1.0;
      w[i][j] = ex * okc[j];
      x[i][j] = mm[i * kNMM + j] * inv[j];
      sh += w[i][j] * x[i][j];
      ch += w[i][j];
    }
    sum[h] += sh;
    cnt[h] += ch;
  }
  const double mean[3] = {(sum[0] + sum[1]) / (cnt[0] + cnt[1]), sum[0] / cnt[0], sum[1] / cnt[1]};
  double ss[3] = {0.0, 0.0, 0.0};
  for (int i = 0; i < kNPos; ++i) {
    const int h = i >= kNHalf;
    const double mh = mean[1 + h];
    double s0 = 0.0, s1 = 0.0;
    for (int j = 0; j < kNMM; ++j) {
      const double d0 = x[i][j] - mean[0], d1 = x[i][j] - mh;
      s0 += w[i][j] * d0 * d0;
      s1 += w[i][j] * d1 * d1;
    }
    ss[0] += s0;
    ss[1 + h] += s1;
  }
  const double n3[3] = {cnt[0] + cnt[1], cnt[0], cnt[1]};
  for (int r = 0; r < 3; ++r) out3[r] = n3[r] > 0.0 ? __builtin_sqrt(ss[r] / n3[r]) : __builtin_nan("");
}
}  // namespace

extern "C" int mdi_noise(const uint32_t* mm, int64_t n_taxa, int n_threads, double* out3) {
  if (n_taxa < 0 || (n_taxa > 0 && (!mm || !out3))) return MDI_E_ARG;
  if (n_taxa == 0) return 0;
  int nt = n_threads > 0 ? n_threads : mdi_default_threads();
  if (nt < 1) nt = 1;
  if ((int64_t)nt > (n_taxa + 511) / 512) nt = (int)((n_taxa + 511) / 512);
  std::vector<std::thread> pool;
  const int64_t per = (n_taxa + nt - 1) / nt;
  for (int k = 0; k < nt; ++k) {
    const int64_t a = k * per, b = std::min(n_taxa, a + per);
    if (a >= b) break;
    pool.emplace_back([=] {
      for (int64_t t = a; t < b; ++t) noise_one(mm + t * kNPos * kNMM, out3 + 3 * t);
    });
  }
  for (auto& th : pool) th.join();
  return 0;
}
