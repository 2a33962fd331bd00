// karlin_ref.cpp — TEST INFRASTRUCTURE ONLY (SURVEY.md §8 f4 parity pin).
//
// Prints the reference's own general Karlin-Altschul results for the matrix
// files given: Statistics::CalculateUngappedIdealKarlinParameters
// (statistics.cpp:100-112 -> karlin.cpp BlastKarlinBlkCalc) and
// BlastComputeLengthAdjustment (karlin.cpp:393-476) for a fixed set of
// (query length, DB length, DB sequences). Built by oracle/Makefile from the
// reference sources where they lie (oracle/_ref/karlin_ref); its output is
// committed as tests/golden/karlin_golden.json by tests/golden/make_karlin_golden.py.
// A path that cannot be opened gives the reference's built-in BLOSUM62.
#include <cmath>
#include <cstdio>
#include <cstring>

#include "karlin.h"
#include "score_matrix_reader.h"
#include "statistics.h"

static unsigned FloatBits(float f) {
  unsigned u;
  std::memcpy(&u, &f, 4);
  return u;
}

int main(int argc, char **argv) {
  static const int kCases[][3] = {{127, 10000000, 33000}, {75, 381, 4}, {300, 5000000, 16000},
                                  {20, 1000000, 3000}, {1, 376, 4}, {1000, 100, 1}};
  std::printf("[\n");
  for (int a = 1; a < argc; ++a) {
    ScoreMatrixReader reader;
    ScoreMatrix *m = reader.Read(argv[a]);
    Statistics st;
    KarlinParameters p;
    st.CalculateUngappedIdealKarlinParameters(*m, &p);
    std::printf("%s{\"path\": \"%s\", \"name\": \"%s\", \"lambda\": %u, \"K\": %u, \"H\": %u, \"logK\": %u, \"adjust\": [",
                a > 1 ? "," : "", argv[a], m->GetName().c_str(), FloatBits(p.lambda), FloatBits(p.K), FloatBits(p.H),
                FloatBits(logf(p.K)));
    if (!(p.K > 0.f) || !(p.H > 0.f)) {  // no parameters: no adjustment to pin
      std::printf("]}\n");
      delete m;
      continue;
    }
    for (size_t c = 0; c < sizeof(kCases) / sizeof(kCases[0]); ++c) {
      int adj = -1;
      const int rc = BlastComputeLengthAdjustment(p.K, logf(p.K), 1.0f / p.H, 0.0f, kCases[c][0],
                                                  (uint32_t)kCases[c][1], kCases[c][2], &adj);
      std::printf("%s[%d, %d, %d, %d, %d]", c ? ", " : "", kCases[c][0], kCases[c][1], kCases[c][2], adj, rc);
    }
    std::printf("]}\n");
    delete m;
  }
  std::printf("]\n");
  return 0;
}
