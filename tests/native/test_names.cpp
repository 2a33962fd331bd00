// NameTable / ReadNameLines (ghostm_amd/csrc/formats.cpp) against the
// reference's getline reading (query_reader.cpp, ReadNameLines' fallback):
// complete files, files with fewer lines than sequences, an unterminated last
// line, empty names, a missing file, and slices of each.
#include <cstdio>
#include <fstream>
#include <random>
#include <string>
#include <vector>

#include "../../ghostm_amd/csrc/formats.h"

static std::vector<std::string> Getline(const std::string &path, uint32_t n) {
  std::vector<std::string> out(n);
  std::ifstream f(path.c_str());
  if (!f) return out;
  std::string line;
  for (uint32_t i = 0; i < n && !f.eof(); ++i) {
    std::getline(f, line);
    out[i] = line;
  }
  return out;
}

int main(int argc, char **argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  std::mt19937 rng(3);
  int bad = 0, cases = 0;
  for (int t = 0; t < 300; ++t) {
    const uint32_t lines = rng() % 200;
    std::string text;
    for (uint32_t i = 0; i < lines; ++i) {
      const uint32_t len = rng() % 5 == 0 ? 0 : rng() % 20;
      for (uint32_t k = 0; k < len; ++k) text.push_back((char)('a' + rng() % 26));
      if (i + 1 < lines || rng() % 2) text.push_back('\n');  // sometimes unterminated
    }
    const std::string path = dir + "/names_" + std::to_string(t) + ".nam";
    { std::ofstream o(path.c_str(), std::ios::binary); o << text; }
    const uint32_t n = rng() % 3 == 0 ? lines + rng() % 5 : (lines ? rng() % lines : 0);
    const std::vector<std::string> want = Getline(t % 50 == 7 ? dir + "/missing.nam" : path, n);
    const ghostm::NameTable got = ghostm::ReadNameLines(t % 50 == 7 ? dir + "/missing.nam" : path, n, nullptr);
    ++cases;
    if (got.size() != n) { printf("case %d: %zu names, want %u\n", t, got.size(), n); ++bad; continue; }
    for (uint32_t i = 0; i < n; ++i)
      if (std::string(got[i]) != want[i]) { printf("case %d name %u differs\n", t, i); ++bad; break; }
    if (n) {
      const uint32_t i0 = rng() % n, m = rng() % (n - i0 + 1);
      const ghostm::NameTable s = got.Slice(i0, m);
      for (uint32_t k = 0; k < m; ++k)
        if (std::string(s[k]) != want[i0 + k]) { printf("case %d slice differs\n", t); ++bad; break; }
      ghostm::NameTable grown = s;  // names added one by one after a slice
      grown.push_back("extra");
      if (grown.size() != m + 1 || std::string(grown[m]) != "extra" || (m && std::string(grown[0]) != want[i0])) {
        printf("case %d push_back differs\n", t);
        ++bad;
      }
    }
  }
  printf("%d cases, %d mismatches\n", cases, bad);
  return bad != 0;
}
