// scoring.h — substitution matrix and Karlin–Altschul statistics of the `aln`
// path.
//   ScoreMatrix / reader: reference score_matrix.cpp:33-48,
//                         score_matrix_reader.cpp:44-113 (NCBI text, built-in
//                         BLOSUM62 when the -M file cannot be opened)
//   Statistics:           statistics.cpp:40-59 (bits, E-value, search space) and
//                         the gapped-parameter table statistics.cpp:134-146
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace ghostm {

struct ScoreMatrix {
  std::string name;        // file basename, or "BLOSUM62" for the built-in one
  std::vector<int> m;      // 32 x 32, m[db_code * 32 + query_code]
  int highest = 0, lowest = 0;
  int At(int db_code, int query_code) const { return m[db_code * 32 + query_code]; }
};

// Read an NCBI-layout matrix file; falls back to built-in BLOSUM62 when the path
// cannot be opened (same rule and the same parsing quirks as the reference).
ScoreMatrix ReadScoreMatrix(const std::string &path);
ScoreMatrix BuiltinBlosum62();

struct KarlinParams {
  float lambda = 0.f, K = 0.f, H = 0.f;
};

// statistics.cpp:134-146 — only BLOSUM62 11/1 and PAM30 9/1 are known; any other
// combination throws "error: not support score option".
KarlinParams GappedKarlinParams(const ScoreMatrix &mx, int open_gap, int extend_gap);

// General ungapped parameters for any matrix (karlin_params.cpp): the reference's
// Statistics::CalculateUngappedIdealKarlinParameters (statistics.cpp:100-112) with
// BLAST's routines (karlin.cpp:16-324), Robinson & Robinson background.
KarlinParams UngappedKarlinParams(const ScoreMatrix &mx);
// BlastComputeLengthAdjustment (karlin.cpp:393-476); returns 0 when converged.
int LengthAdjustment(float K, float logK, float alpha_d_lambda, float beta, int query_length, uint32_t db_length,
                     int db_num_seqs, int *adjustment);

// Float/double arithmetic exactly as the reference (A.7 of SURVEY.md):
//   bits = ((float)s * lambda - logf(K)) / (float)log(2.0)
//   E    = (float)((double)((float)space * K) * exp(-1.0 * s * (double)lambda))
struct EvalueCalculator {
  KarlinParams p;
  float log_k = 0.f, log2_f = 0.f;
  explicit EvalueCalculator(const KarlinParams &params);
  float Bits(int score) const;
  float Evalue(int score, uint64_t search_space) const;
};

}  // namespace ghostm
