// synth.cpp — `ghostm synth`: deterministic synthetic FASTA for the benchmark
// configurations of SURVEY.md §8(d2) (the reference ships no large inputs;
// testset/large_queries.fasta is absent).
//   DB subjects: length U[smin, smax], residues i.i.d. from the Robinson
//     background frequencies the reference uses for its statistics
//     (statistics.cpp:74-93).
//   Queries: length U[qmin, qmax]; a fraction `homolog` are substrings of random
//     subjects with `subst` uniform substitutions, the rest background-random.
//   DNA reads (-t dna): length -l nt; a fraction `homolog` back-translate a random
//     subject segment (random synonymous codons, `subst` of them mutated), the rest
//     are uniform random bases.
//   -D FASTA: queries sample the subjects of an existing FASTA instead (the
//     BASELINE config-2 substitute: testset/db.fasta, whose large_queries.fasta is
//     absent from the reference); substrings are clipped to the subject length.
// RNG: splitmix64, so the files are identical on every host.
#include <getopt.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace ghostm {

namespace {

struct SplitMix64 {
  uint64_t s;
  explicit SplitMix64(uint64_t seed) : s(seed) {}
  uint64_t Next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double Uniform() { return (Next() >> 11) * (1.0 / 9007199254740992.0); }
  uint32_t Range(uint32_t lo, uint32_t hi) {  // inclusive
    return lo + (uint32_t)(Next() % (uint64_t)(hi - lo + 1));
  }
};

const char kLetters[] = "ARNDCQEGHILKMFPSTWYV";
// Robinson & Robinson background (per mille), in kLetters order.
const double kFreq[20] = {78.05, 51.29, 44.87, 53.64, 19.25, 42.64, 62.95, 73.77, 21.99, 51.42,
                          90.19, 57.44, 22.43, 38.56, 52.03, 71.20, 58.41, 13.30, 32.16, 64.41};

struct Background {
  double cdf[20];
  Background() {
    double s = 0;
    for (double f : kFreq) s += f;
    double acc = 0;
    for (int i = 0; i < 20; ++i) {
      acc += kFreq[i] / s;
      cdf[i] = acc;
    }
    cdf[19] = 1.0;
  }
  char Draw(SplitMix64 &r) const {
    const double u = r.Uniform();
    for (int i = 0; i < 20; ++i)
      if (u < cdf[i]) return kLetters[i];
    return kLetters[19];
  }
};

// one codon per amino acid letter of kLetters (any synonymous choice works)
const char *const kCodonsFor[20] = {"GCT", "CGT", "AAT", "GAT", "TGT", "CAA", "GAA", "GGT", "CAT", "ATT",
                                    "CTG", "AAA", "ATG", "TTT", "CCG", "TCT", "ACC", "TGG", "TAT", "GTG"};

void WriteFasta(FILE *f, const std::string &name, const std::string &seq) {
  fprintf(f, ">%s\n", name.c_str());
  for (size_t p = 0; p < seq.size(); p += 60) {
    const size_t n = std::min<size_t>(60, seq.size() - p);
    fwrite(seq.data() + p, 1, n, f);
    fputc('\n', f);
  }
}

}  // namespace

// ghostm synth -d DB.fasta -q Q.fasta [-n nq] [-N db_residues] [-s seed]
//              [-a qmin] [-b qmax] [-m smin] [-x smax] [-h homolog] [-u subst]
//              [-p qprefix] [-f first_query_index]
int SynthMain(int argc, char **argv) {
  std::string db_path, q_path, qname_prefix = "q";
  uint64_t nq = 1000, db_res = 1000000, seed = 3, first = 0;
  uint32_t qmin = 200, qmax = 400, smin = 100, smax = 600;
  double homolog = 0.8, subst = 0.15;
  bool dna = false;
  uint32_t read_len = 150;
  std::string subjects_from;
  optind = 1;
  int c;
  while ((c = getopt(argc, argv, "d:q:n:N:s:a:b:m:x:h:u:p:f:t:l:D:")) >= 0) {
    switch (c) {
      case 'd': db_path = optarg; break;
      case 'q': q_path = optarg; break;
      case 'n': nq = strtoull(optarg, nullptr, 10); break;
      case 'N': db_res = strtoull(optarg, nullptr, 10); break;
      case 's': seed = strtoull(optarg, nullptr, 10); break;
      case 'a': qmin = atoi(optarg); break;
      case 'b': qmax = atoi(optarg); break;
      case 'm': smin = atoi(optarg); break;
      case 'x': smax = atoi(optarg); break;
      case 'h': homolog = atof(optarg); break;
      case 'u': subst = atof(optarg); break;
      case 'p': qname_prefix = optarg; break;
      case 'f': first = strtoull(optarg, nullptr, 10); break;
      case 't': dna = strcmp(optarg, "dna") == 0; break;
      case 'l': read_len = atoi(optarg); break;
      case 'D': subjects_from = optarg; break;
      default: throw std::invalid_argument("synth: bad option");
    }
  }
  if (qmin < 1 || qmax < qmin || smin < 1 || smax < smin)
    throw std::invalid_argument("synth: bad length range");
  const Background bg;
  // the database is a function of (seed, db_res, lengths) only
  SplitMix64 rdb(seed * 1000003ull + 17);
  std::vector<std::string> subjects;
  uint64_t total = 0;
  if (!subjects_from.empty()) {
    FILE *f = fopen(subjects_from.c_str(), "r");
    if (!f) throw std::runtime_error("synth: cannot read " + subjects_from);
    char line[4096];
    while (fgets(line, sizeof(line), f)) {
      if (line[0] == '>') {
        subjects.emplace_back();
        continue;
      }
      if (subjects.empty()) continue;
      for (const char *p = line; *p; ++p)
        if ((*p >= 'A' && *p <= 'Z') || (*p >= 'a' && *p <= 'z') || *p == '*') subjects.back().push_back(*p);
    }
    fclose(f);
    while (!subjects.empty() && subjects.back().empty()) subjects.pop_back();
    if (subjects.empty()) throw std::runtime_error("synth: no subjects in " + subjects_from);
    db_res = 0;  // no generated subjects
  }
  while (total < db_res) {
    const uint32_t len = rdb.Range(smin, smax);
    std::string s(len, 'A');
    for (auto &ch : s) ch = bg.Draw(rdb);
    total += len;
    subjects.push_back(std::move(s));
  }
  if (!db_path.empty()) {
    FILE *f = fopen(db_path.c_str(), "w");
    if (!f) throw std::runtime_error("synth: cannot write " + db_path);
    for (size_t i = 0; i < subjects.size(); ++i) WriteFasta(f, "s" + std::to_string(i), subjects[i]);
    fclose(f);
  }
  if (!q_path.empty()) {
    FILE *f = fopen(q_path.c_str(), "w");
    if (!f) throw std::runtime_error("synth: cannot write " + q_path);
    for (uint64_t k = 0; k < nq; ++k) {
      const uint64_t qi = first + k;
      SplitMix64 r(seed * 0x100000001B3ull + qi * 0x9E3779B97F4A7C15ull + 1);
      std::string q;
      if (dna) {
        static const char kBases[] = "ACGT";
        if (r.Uniform() < homolog) {
          const std::string &s = subjects[r.Next() % subjects.size()];
          const uint32_t aa = std::min<uint32_t>((read_len + 2) / 3, (uint32_t)s.size());
          const uint32_t at = r.Range(0, (uint32_t)s.size() - aa);
          for (uint32_t k = 0; k < aa; ++k) {
            const char *cod = kCodonsFor[strchr(kLetters, s[at + k]) - kLetters];
            for (int b = 0; b < 3; ++b)
              q.push_back(r.Uniform() < subst / 3 ? kBases[r.Next() % 4] : cod[b]);
          }
          q.resize(read_len, 'A');
          if (r.Uniform() < 0.5) {  // reverse complement half of them
            std::string rc(q.rbegin(), q.rend());
            for (auto &ch : rc) ch = ch == 'A' ? 'T' : ch == 'C' ? 'G' : ch == 'G' ? 'C' : 'A';
            q.swap(rc);
          }
        } else {
          q.resize(read_len);
          for (auto &ch : q) ch = kBases[r.Next() % 4];
        }
        WriteFasta(f, qname_prefix + std::to_string(qi), q);
        continue;
      }
      const uint32_t len = r.Range(qmin, qmax);
      if (r.Uniform() < homolog) {
        const std::string &s = subjects[r.Next() % subjects.size()];
        const uint32_t take = std::min<uint32_t>(len, (uint32_t)s.size());
        const uint32_t at = r.Range(0, (uint32_t)s.size() - take);
        q = s.substr(at, take);
        for (auto &ch : q)
          if (r.Uniform() < subst) ch = kLetters[r.Next() % 20];
      } else {
        q.assign(len, 'A');
        for (auto &ch : q) ch = bg.Draw(r);
      }
      WriteFasta(f, qname_prefix + std::to_string(qi), q);
    }
    fclose(f);
  }
  return 0;
}

}  // namespace ghostm
