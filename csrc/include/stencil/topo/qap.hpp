#pragma once
// Quadratic assignment problem solvers used to place sub-domains onto GPUs.
// cost(f) = sum_{a,b} w(a,b) * d(f(a), f(b)), with 0 * inf := 0.
// Parity: reference include/stencil/qap.hpp
//   solve        exhaustive permutation search     qap.hpp:50-75
//   solve_catch  best-single-swap local search      qap.hpp:77-172
// Differences (by design): `solve` is exhaustive only up to n<=10 and falls back to
// solve_catch beyond (10! = 3.6M perms x n^2); the swap search uses the same O(n) delta update.
#include <algorithm>
#include <cmath>
#include <numeric>
#include <vector>

#include "stencil/topo/mat2d.hpp"

namespace qap {
namespace detail {
inline double cost_product(double we, double de) { return (we == 0 || de == 0) ? 0.0 : we * de; }

inline double cost(const Mat2D<double> &w, const Mat2D<double> &d, const std::vector<size_t> &f) {
  double ret = 0;
  const size_t n = f.size();
  for (size_t a = 0; a < n; ++a)
    for (size_t b = 0; b < n; ++b) ret += cost_product(w.at(a, b), d.at(f[a], f[b]));
  return ret;
}

// add sign * (contribution of rows/cols i and j, without double counting) to c, term by term
inline void pair_terms(double &c, double sign, const Mat2D<double> &w, const Mat2D<double> &d,
                       const std::vector<size_t> &f, size_t i, size_t j) {
  const size_t n = f.size();
  for (size_t k = 0; k < n; ++k) {
    c += sign * cost_product(w.at(i, k), d.at(f[i], f[k]));
    c += sign * cost_product(w.at(j, k), d.at(f[j], f[k]));
    if (k != i && k != j) {
      c += sign * cost_product(w.at(k, i), d.at(f[k], f[i]));
      c += sign * cost_product(w.at(k, j), d.at(f[k], f[j]));
    }
  }
}
} // namespace detail

inline std::vector<size_t> solve_catch(const Mat2D<double> &w, const Mat2D<double> &d, double *costp = nullptr) {
  const size_t n = w.rows();
  std::vector<size_t> best(n);
  std::iota(best.begin(), best.end(), 0);
  double bestCost = detail::cost(w, d, best);
  bool improved = true;
  // incremental costs carry rounding error: demand a strict relative improvement and re-anchor on the exact cost,
  // so two assignments whose costs differ only by rounding cannot swap back and forth forever
  size_t rounds = 0;
  while (improved && rounds++ < 100 * n * n + 100) {
    improved = false;
    std::vector<size_t> imprF = best;
    double imprCost = bestCost;
    for (size_t i = 0; i < n; ++i) {
      for (size_t j = i + 1; j < n; ++j) {
        std::vector<size_t> f = best;
        double c = bestCost;
        detail::pair_terms(c, -1.0, w, d, f, i, j);
        std::swap(f[i], f[j]);
        detail::pair_terms(c, 1.0, w, d, f, i, j);
        if (c < imprCost - 1e-12 * std::fabs(imprCost)) {
          imprF = f;
          imprCost = c;
          improved = true;
        }
      }
    }
    if (improved) {
      best = imprF;
      bestCost = detail::cost(w, d, best);
    }
  }
  if (costp) *costp = bestCost;
  return best;
}

// Exhaustive search in lexicographic permutation order; the first strictly-better
// permutation wins ties, so the result is deterministic (identity on a uniform mesh).
inline std::vector<size_t> solve(const Mat2D<double> &w, const Mat2D<double> &d, double *costp = nullptr) {
  const size_t n = w.rows();
  if (n > 10) return solve_catch(w, d, costp);
  std::vector<size_t> f(n);
  std::iota(f.begin(), f.end(), 0);
  std::vector<size_t> best = f;
  double bestCost = detail::cost(w, d, f);
  do {
    const double c = detail::cost(w, d, f);
    if (c < bestCost) {
      bestCost = c;
      best = f;
    }
  } while (std::next_permutation(f.begin(), f.end()));
  if (costp) *costp = bestCost;
  return best;
}
} // namespace qap
