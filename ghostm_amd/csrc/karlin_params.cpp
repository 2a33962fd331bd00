// karlin_params.cpp — general (ungapped) Karlin–Altschul parameters for any
// substitution matrix.
//
// The reference `aln` path knows only two gapped parameter sets
// (statistics.cpp:134-146) and throws for every other matrix/gap combination.
// Its vendored karlin.cpp (BLAST's Karlin–Altschul routines) and
// Statistics::CalculateUngappedIdealKarlinParameters (statistics.cpp:100-112)
// compute ungapped lambda, K and H from a matrix and the Robinson & Robinson
// background; nothing on the `aln` path calls them. This file restates them
// (same double arithmetic, same float narrowing between the steps, so the
// results are bit-identical, tests/test_karlin.py) for E-values with other
// matrices (GHOSTM_KARLIN=ungapped, aligner.cpp), and restates
// BlastComputeLengthAdjustment (karlin.cpp:393-476) for callers that want the
// edge-effect correction.
//
//   ScoreDistribution  statistics.cpp:148-181 (CalculateScoreProbabilities)
//   Lambda             karlin.cpp:187-289 (Newton-Raphson, bisection fallback)
//   Entropy            karlin.cpp:297-324 (H from lambda)
//   KParameter         karlin.cpp:68-180 (K from lambda and H)
//
// The routines restated here carry this notice in the reference
// (karlin.cpp:1-4), retained as it asks:
//   karlin.c
//   Copyright (c) 2005, Michael Cameron
//   Permission to use this code is freely granted under the BSD license
//   agreement, provided that this statement is retained.
#include <cmath>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../include/ghostm_hip.h"
#include "scoring.h"

namespace ghostm {

void SetLastErrorMessage(const std::string &m);

namespace {

constexpr int kScoreFloor = -10000, kScoreCeil = 1000;  // the routines' accepted score range
constexpr double kLambdaStart = 0.5, kLambdaTol = 1e-5;
constexpr int kBisectSteps = 17;
constexpr double kKSumTol = 0.01;
constexpr int kKTerms = 100;

// Score probabilities indexed by score s in [lo, hi]: prob[s - lo].
struct Distribution {
  int lo = 0, hi = 0;
  std::vector<double> prob;
  double At(int s) const { return prob[(size_t)(s - lo)]; }
};

bool RangeUsable(int lo, int hi) {
  return lo < 0 && hi > 0 && lo >= kScoreFloor && hi <= kScoreCeil && hi - lo <= kScoreCeil - kScoreFloor;
}

// Robinson & Robinson residue frequencies over codes 0..24 (statistics.cpp:73-94)
std::vector<double> Background() {
  // per code (A R N D C Q E G H I L K M F P S T W Y V; B J Z X * absent)
  static const double kPerMille[20] = {78.05, 51.29, 44.87, 53.64, 19.25, 42.64, 62.95, 73.77, 21.99, 51.42,
                                       90.19, 57.44, 22.43, 38.56, 52.03, 71.20, 58.41, 13.30, 32.16, 64.41};
  std::vector<double> f(25, 0.0);
  double total = 0.0;
  for (int c = 0; c < 20; ++c) f[c] = kPerMille[c];
  for (int c = 0; c < 25; ++c) total += f[c];
  for (int c = 0; c < 25; ++c) f[c] = f[c] / total * 1.0;
  return f;
}

Distribution ScoreDistribution(const ScoreMatrix &mx, const std::vector<double> &f1, const std::vector<double> &f2) {
  Distribution d;
  d.lo = mx.lowest;
  d.hi = mx.highest;
  d.prob.assign((size_t)(d.hi - d.lo + 1), 0.0);
  for (int a = 0; a < 25; ++a)
    for (int b = 0; b < 25; ++b) d.prob[(size_t)(mx.m[a * 32 + b] - d.lo)] += f1[a] * f2[b];
  double norm = 0.0;
  for (double p : d.prob)
    if (p > 0.0) norm += p;
  if (norm <= 0.0) throw std::invalid_argument("sum of score frequencies is 0");
  for (double &p : d.prob)
    if (p > 0.0) p /= norm;
  return d;
}

// sum_s p(s) e^{x s} - 1 and its derivative, by powers of e^x from e^{x lo}
// (the reference's running product), or exp per score when that underflows
double MomentMinusOne(const Distribution &d, double x, double *slope) {
  const double ex = exp(x);
  double run = pow(ex, d.lo - 1);
  double sum = -1.0, d1 = 0.0;
  for (int s = d.lo; s <= d.hi; ++s) {
    run *= ex;
    const double t = d.At(s) * run;
    sum += t;
    d1 += t * s;
  }
  if (slope) *slope = d1;
  return sum;
}

double LambdaBisect(const Distribution &d) {
  if (!RangeUsable(d.lo, d.hi)) return -1.0;
  auto moment = [&](double x) {
    const double ex = exp(x);
    double run = pow(ex, d.lo - 1), sum = 0.0;
    if (run > 0.0) {
      for (int s = d.lo; s <= d.hi; ++s) sum += d.At(s) * (run *= ex);
    } else {
      for (int s = d.lo; s <= d.hi; ++s) sum += d.At(s) * exp(x * s);
    }
    return sum;
  };
  double below = 0.0, above = kLambdaStart;
  for (;;) {  // double the upper end until the moment reaches 1
    above *= 2;
    if (moment(above) >= 1.0) break;
    below = above;
  }
  for (int k = 0; k < kBisectSteps; ++k) {
    const double mid = (below + above) / 2.;
    if (moment(mid) > 1.0) above = mid;
    else below = mid;
  }
  return (below + above) / 2.;
}

double Lambda(const Distribution &d) {
  if (!RangeUsable(d.lo, d.hi)) return -1.0;
  double x = kLambdaStart;
  for (int it = 0; it < 20; ++it) {
    if (x < 0.01) break;
    if (pow(exp(x), d.lo - 1) == 0.) break;
    double slope = 0.0;
    const double f = MomentMinusOne(d, x, &slope);
    const double step = f / slope;
    x -= step;
    if (std::fabs(step / x) < kLambdaTol) {
      if (x > kLambdaTol) return x;  // not the trivial root at 0
      break;
    }
  }
  return LambdaBisect(d);
}

double Entropy(const Distribution &d, double lambda) {
  if (lambda < 0.) return -1.;
  if (!RangeUsable(d.lo, d.hi)) return -1.;
  const double el = exp(lambda);
  double run = pow(el, d.lo - 1), av = 0.0;
  if (run > 0.) {
    for (int s = d.lo; s <= d.hi; ++s) av += d.At(s) * s * (run *= el);
  } else {
    for (int s = d.lo; s <= d.hi; ++s) av += d.At(s) * s * exp(lambda * s);
  }
  return lambda * av;
}

long Gcd(long a, long b) {
  b = b < 0 ? -b : b;
  if (b > a) std::swap(a, b);
  while (b != 0) {
    const long r = a % b;
    a = b;
    b = r;
  }
  return a;
}

// K from the distribution of the sum of i.i.d. scores (Karlin & Altschul 1990):
// the term for j steps needs the j-fold convolution of p; terms stop below
// kKSumTol (or after kKTerms), then a geometric tail is added.
double KParameter(const Distribution &d, double lambda, double H) {
  if (lambda <= 0. || H <= 0.) return -1.;
  const int lo = d.lo, hi = d.hi, range = hi - lo;
  const double av = H / lambda;
  const double el = exp(lambda);
  if (lo == -1 || hi == 1) return av * (1.0 - 1. / el);
  if (kKTerms * range + 1 > kKTerms * (kScoreCeil - kScoreFloor) + 1) return -1.;
  // conv[t] = probability that the j-step sum equals (lo * j + t)
  std::vector<double> conv((size_t)(kKTerms * range + 1), 0.0);
  const double *p = d.prob.data();  // p[t] = prob of score lo + t
  double term = 1.0, prev = 1.0, prev2 = 1.0, total = 0.;
  int span_lo = 0, span_hi = 0, j = 0;
  conv[0] = 1.;
  for (; j < kKTerms && term > kKSumTol; total += term /= ++j) {
    span_lo += lo;
    span_hi += hi;
    // next convolution in place, from the top: new[t] = sum over k of
    // old[t - k] p[k], k ascending over the offsets that stay inside both
    int first = range, last = range;
    for (int t = span_hi - span_lo; t >= 0; --t) {
      double acc = 0.;
      for (int k = first; k <= last; ++k) acc += conv[(size_t)(t - k)] * p[k];
      conv[(size_t)t] = acc;
      if (first) --first;
      if (t <= range) --last;
    }
    // the j-step sum's expectation of e^{lambda s} over s < 0, plus P(s >= 0)
    double pw = pow(el, span_lo - 1);
    double next = 0.;
    int t = 0;
    for (int s = span_lo; s != 0; ++s, ++t) {
      pw *= el;
      next += conv[(size_t)t] * pw;
    }
    for (int s = 0; s <= span_hi; ++s, ++t) next += conv[(size_t)t];
    prev2 = prev;
    prev = next;
    term = next;
  }
  const double ratio = prev / prev2;
  if (ratio >= (1.0 - kKSumTol * 0.001)) return -1.;
  const double tail_tol = kKSumTol * 0.01;
  while (term > tail_tol) {
    prev *= ratio;
    total += term = prev / ++j;
  }
  // delta: the gcd of the scores that occur (PNAS 87, appendix)
  long g = -lo;
  for (int i = 1; i <= range && g > 1; ++i)
    if (p[i]) g = Gcd(g, i);
  if (g * el > 0.05) return g * exp((double)-2.0 * total) / (av * (1.0 - pow(el, -g)));
  return -g * exp((double)-2.0 * total) / (av * (exp(-g * lambda) - 1));
}

}  // namespace

// Statistics::CalculateUngappedIdealKarlinParameters + BlastKarlinBlkCalc:
// lambda, then H from the float lambda, then K from both floats.
KarlinParams UngappedKarlinParams(const ScoreMatrix &mx) {
  const std::vector<double> bg = Background();
  const Distribution d = ScoreDistribution(mx, bg, bg);
  KarlinParams k;
  k.lambda = (float)Lambda(d);
  k.H = (float)Entropy(d, k.lambda);
  k.K = (float)KParameter(d, k.lambda, k.H);
  return k;
}

// BlastComputeLengthAdjustment: the largest integer below the fixed point of
// ell = alpha/lambda (log K + log((m - ell)(n - N ell))) + beta, bracketed and
// iterated at most 20 times; returns 0 when it converged.
int LengthAdjustment(float K, float logK, float alpha_d_lambda, float beta, int query_length, uint32_t db_length,
                     int db_num_seqs, int *adjustment) {
  const double m = query_length, n = db_length, N = db_num_seqs;
  const double c = n * m - (m > n ? m : n) / K;
  if (c < 0) {
    *adjustment = 0;
    return 1;
  }
  const double mb = m * N + n;
  double top = 2 * c / (mb + sqrt(mb * mb - 4 * N * c)), bottom = 0, next = 0;
  bool converged = false;
  for (int it = 1; it <= 20; ++it) {
    const double ell = next;
    const double proposal = alpha_d_lambda * (logK + log((m - ell) * (n - N * ell))) + beta;
    if (proposal >= ell) {
      bottom = ell;
      if (proposal - bottom <= 1.0) {
        converged = true;
        break;
      }
      if (bottom == top) break;
    } else {
      top = ell;
    }
    next = (bottom <= proposal && proposal <= top) ? proposal : (it == 1 ? top : (bottom + top) / 2);
  }
  *adjustment = (int)bottom;
  if (converged) {
    const double up = ceil(bottom);
    if (up <= top && alpha_d_lambda * (logK + log((m - up) * (n - N * up))) + beta >= up) *adjustment = (int)up;
  }
  return converged ? 0 : 1;
}

}  // namespace ghostm

extern "C" int GhostmKarlinUngapped(const int score_matrix[], float *lambda, float *K, float *H) {
  try {
    if (!score_matrix || !lambda || !K || !H) throw std::invalid_argument("null argument");
    ghostm::ScoreMatrix mx;
    mx.m.assign(score_matrix, score_matrix + 32 * 32);
    for (int v : mx.m) {
      if (v > mx.highest) mx.highest = v;
      if (v < mx.lowest) mx.lowest = v;
    }
    const ghostm::KarlinParams p = ghostm::UngappedKarlinParams(mx);
    *lambda = p.lambda;
    *K = p.K;
    *H = p.H;
    return 0;
  } catch (std::exception &e) {
    ghostm::SetLastErrorMessage(e.what());
    return 1;
  }
}

extern "C" int GhostmReadScoreMatrix(const char *path, int score_matrix[]) {
  try {
    if (!path || !score_matrix) throw std::invalid_argument("null argument");
    const ghostm::ScoreMatrix mx = ghostm::ReadScoreMatrix(path);
    for (int i = 0; i < 32 * 32; ++i) score_matrix[i] = mx.m[(size_t)i];
    return 0;
  } catch (std::exception &e) {
    ghostm::SetLastErrorMessage(e.what());
    return 1;
  }
}

extern "C" int GhostmLengthAdjustment(float K, float logK, float alpha_d_lambda, float beta, int query_length,
                                      uint32_t db_length, int db_num_seqs, int *length_adjustment) {
  if (!length_adjustment) return -1;
  return ghostm::LengthAdjustment(K, logK, alpha_d_lambda, beta, query_length, db_length, db_num_seqs,
                                  length_adjustment);
}
