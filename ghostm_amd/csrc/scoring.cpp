// scoring.cpp — see scoring.h.
#include "scoring.h"

#include <cmath>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "common.h"

namespace ghostm {

namespace {

// Standard BLOSUM62 (half-bit units) over A R N D C Q E G H I L K M F P S T W Y V
// B Z X *, in the NCBI layout the reference embeds (score_matrix_reader.cpp:40-42).
const char kBlosum62Text[] =
    "   A  R  N  D  C  Q  E  G  H  I  L  K  M  F  P  S  T  W  Y  V  B  Z  X  *\n"
    "A  4 -1 -2 -2  0 -1 -1  0 -2 -1 -1 -1 -1 -2 -1  1  0 -3 -2  0 -2 -1  0 -4\n"
    "R -1  5  0 -2 -3  1  0 -2  0 -3 -2  2 -1 -3 -2 -1 -1 -3 -2 -3 -1  0 -1 -4\n"
    "N -2  0  6  1 -3  0  0  0  1 -3 -3  0 -2 -3 -2  1  0 -4 -2 -3  3  0 -1 -4\n"
    "D -2 -2  1  6 -3  0  2 -1 -1 -3 -4 -1 -3 -3 -1  0 -1 -4 -3 -3  4  1 -1 -4\n"
    "C  0 -3 -3 -3  9 -3 -4 -3 -3 -1 -1 -3 -1 -2 -3 -1 -1 -2 -2 -1 -3 -3 -2 -4\n"
    "Q -1  1  0  0 -3  5  2 -2  0 -3 -2  1  0 -3 -1  0 -1 -2 -1 -2  0  3 -1 -4\n"
    "E -1  0  0  2 -4  2  5 -2  0 -3 -3  1 -2 -3 -1  0 -1 -3 -2 -2  1  4 -1 -4\n"
    "G  0 -2  0 -1 -3 -2 -2  6 -2 -4 -4 -2 -3 -3 -2  0 -2 -2 -3 -3 -1 -2 -1 -4\n"
    "H -2  0  1 -1 -3  0  0 -2  8 -3 -3 -1 -2 -1 -2 -1 -2 -2  2 -3  0  0 -1 -4\n"
    "I -1 -3 -3 -3 -1 -3 -3 -4 -3  4  2 -3  1  0 -3 -2 -1 -3 -1  3 -3 -3 -1 -4\n"
    "L -1 -2 -3 -4 -1 -2 -3 -4 -3  2  4 -2  2  0 -3 -2 -1 -2 -1  1 -4 -3 -1 -4\n"
    "K -1  2  0 -1 -3  1  1 -2 -1 -3 -2  5 -1 -3 -1  0 -1 -3 -2 -2  0  1 -1 -4\n"
    "M -1 -1 -2 -3 -1  0 -2 -3 -2  1  2 -1  5  0 -2 -1 -1 -1 -1  1 -3 -1 -1 -4\n"
    "F -2 -3 -3 -3 -2 -3 -3 -3 -1  0  0 -3  0  6 -4 -2 -2  1  3 -1 -3 -3 -1 -4\n"
    "P -1 -2 -2 -1 -3 -1 -1 -2 -2 -3 -3 -1 -2 -4  7 -1 -1 -4 -3 -2 -2 -1 -2 -4\n"
    "S  1 -1  1  0 -1  0  0  0 -1 -2 -2  0 -1 -2 -1  4  1 -3 -2 -2  0  0  0 -4\n"
    "T  0 -1  0 -1 -1 -1 -1 -2 -2 -1 -1 -1 -1 -2 -1  1  5 -2 -2  0 -1 -1  0 -4\n"
    "W -3 -3 -4 -4 -2 -2 -3 -2 -2 -3 -2 -3 -1  1 -4 -3 -2 11  2 -3 -4 -3 -2 -4\n"
    "Y -2 -2 -2 -3 -2 -1 -2 -3  2 -1 -1 -2 -1  3 -3 -2 -2  2  7 -1 -3 -2 -1 -4\n"
    "V  0 -3 -3 -3 -1 -2 -2 -3 -3  3  1 -2  1 -1 -2 -2  0 -3 -1  4 -3 -2 -1 -4\n"
    "B -2 -1  3  4 -3  0  1 -1  0 -3 -4  0 -3 -3 -2  0 -1 -4 -3 -3  4  1 -1 -4\n"
    "Z -1  0  0  1 -3  3  4 -2  0 -3 -3  1 -1 -3 -1  0 -1 -3 -2 -2  1  4 -1 -4\n"
    "X  0 -1 -1 -1 -2 -1 -1 -1 -1 -1 -1 -1 -1 -1 -2  0  0 -2 -1 -1 -1 -1 -1 -4\n"
    "* -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4  1\n";

// Split on single spaces, dropping empty fields (the reader's Split()).
std::vector<std::string> Fields(const std::string &line) {
  std::vector<std::string> out;
  size_t start = 0;
  while (start <= line.size()) {
    size_t stop = line.find(' ', start);
    if (stop == std::string::npos) stop = line.size();
    if (stop > start) out.emplace_back(line, start, stop - start);
    start = stop + 1;
  }
  return out;
}

ScoreMatrix Parse(std::istream &in, const std::string &name) {
  ScoreMatrix mx;
  mx.name = name;
  mx.m.assign(kAlphabet * kAlphabet, 0);
  char heading[kAlphabet] = {0}, row_letter[kAlphabet] = {0};
  int row = 0;  // 0 = heading line, then matrix rows 1..24
  std::string line;
  while (!in.eof()) {
    std::getline(in, line);
    if (line.empty() || line[0] == '#' || row >= kSeqEnd) continue;
    const std::vector<std::string> f = Fields(line);
    for (size_t i = 0; i < f.size() && i < (size_t)kSeqEnd; ++i) {
      if (row == 0) {
        heading[i] = f[i][0];
      } else if (i == 0) {
        row_letter[row - 1] = f[i][0];
      } else {
        mx.m[ProteinCode((unsigned char)row_letter[row - 1]) * kAlphabet +
             ProteinCode((unsigned char)heading[i - 1])] = atoi(f[i].c_str());
      }
    }
    ++row;
  }
  for (int v : mx.m) {
    if (v > mx.highest) mx.highest = v;
    if (v < mx.lowest) mx.lowest = v;
  }
  return mx;
}

}  // namespace

ScoreMatrix BuiltinBlosum62() {
  std::istringstream in(kBlosum62Text);
  return Parse(in, "BLOSUM62");
}

ScoreMatrix ReadScoreMatrix(const std::string &path) {
  std::ifstream in(path.c_str());
  if (!in) return BuiltinBlosum62();
  const size_t slash = path.find_last_of('/');
  return Parse(in, slash == std::string::npos ? path : path.substr(slash + 1));
}

KarlinParams GappedKarlinParams(const ScoreMatrix &mx, int open_gap, int extend_gap) {
  KarlinParams p;
  if (mx.name == "BLOSUM62" && open_gap == -11 && extend_gap == -1) {
    p.lambda = 0.267f; p.K = 0.041f; p.H = 0.14f;
  } else if (mx.name == "PAM30" && open_gap == -9 && extend_gap == -1) {
    p.lambda = 0.294f; p.K = 0.11f; p.H = 0.61f;
  } else {
    throw std::invalid_argument("error: not support score option");
  }
  return p;
}

EvalueCalculator::EvalueCalculator(const KarlinParams &params) : p(params) {
  log_k = logf(p.K);
  log2_f = static_cast<float>(log(2.0));
}

float EvalueCalculator::Bits(int score) const {
  return ((static_cast<float>(score) * p.lambda) - log_k) / log2_f;
}

float EvalueCalculator::Evalue(int score, uint64_t search_space) const {
  const float scaled = (float)search_space * p.K;
  return (float)((double)scaled * exp(static_cast<double>(-1.0 * score * p.lambda)));
}

}  // namespace ghostm
