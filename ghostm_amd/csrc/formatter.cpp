// formatter.cpp — `ghostm db` and `ghostm qry`: FASTA -> the formatted files the
// `aln` hot path reads. Byte-identical to the
// reference formatters:
//   FASTA reader ....... fasta_sequence_reader.cpp:34-86
//   db ................. db_creator.cpp:47-479 (chunking 88-128, concatenation
//                        130-165, k-mer CSR index 167-241, writers 242-355)
//   qry ................ query_creator.cpp:119-517 (chunking 191-240, six-frame
//                        translation 242-324, X padding 388-423)
#include <getopt.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <fstream>
#include <iostream>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/ghostm_hip.h"
#include "common.h"
#include "formats.h"

namespace ghostm {

namespace {

struct FastaRecord {
  std::string name, seq;
};

// One record per Next(); the header line of the following record is kept.
class FastaReader {
 public:
  explicit FastaReader(const std::string &path) : in_(path.c_str()) {}
  bool Next(FastaRecord *r) {
    if (in_.eof()) return false;
    std::string line = held_;
    while (!in_.eof() && (line.empty() || line[0] != '>')) std::getline(in_, line);
    if (in_.eof()) return false;
    if (line.back() == '\r') line.pop_back();
    r->name.clear();
    const size_t p = line.find_first_not_of("> ");
    if (p != std::string::npos) r->name = line.substr(p);
    r->seq.clear();
    while (!in_.eof()) {
      std::getline(in_, line);
      if (line.empty()) continue;
      if (line[0] == '>') break;
      if (line.back() == '\r') line.pop_back();
      if (line.at(line.size() - 1) == '+') line.pop_back();
      r->seq += line;
    }
    held_ = line;
    return true;
  }

 private:
  std::ifstream in_;
  std::string held_;
};

template <class T> void WriteRaw(std::ofstream &f, const T *p, size_t n) {
  f.write(reinterpret_cast<const char *>(p), sizeof(T) * n);
}

void WriteNames(const std::string &path, const std::vector<FastaRecord> &recs) {
  std::ofstream f(path.c_str());
  for (const FastaRecord &r : recs) f << r.name << '\n';
}

}  // namespace

// ------------------------------------------------------------------ db
int DbFormatMain(int argc, char **argv) {
  std::string in_path, out_prefix;
  uint32_t seed = (1u << 4) - 1;
  uint32_t max_concat = 1u << 27;
  int device = -1;  // -D d (extension): build the k-mer index on GPU d
  optind = 1;
  int c;
  while ((c = getopt(argc, argv, "i:o:k:l:D:")) >= 0) {
    switch (c) {
      case 'i': in_path = optarg; break;
      case 'o': out_prefix = optarg; break;
      case 'k': seed = (1u << atoi(optarg)) - 1; break;
      case 'l': max_concat = atoi(optarg) * (1 << 20); break;
      case 'D': device = atoi(optarg); break;
      default: throw std::invalid_argument("");
    }
  }
  const uint32_t seed_len = SeedLength(seed), weight = SeedWeight(seed);
  const uint32_t kcl = (uint32_t)pow(32.0, (double)weight) + 1;
  FastaReader reader(in_path);
  bool pending_valid = false;
  FastaRecord pending;
  uint64_t sum_length = 0;
  for (int chunk = 0;; ++chunk) {
    std::vector<FastaRecord> recs;
    uint32_t sum = 0;
    if (pending_valid) {
      sum = (uint32_t)pending.seq.size() + 1;
      if (sum > max_concat) {
        std::cerr << "error : too small max length." << std::endl;
        return 1;
      }
      recs.push_back(pending);
      pending_valid = false;
    }
    FastaRecord r;
    while (reader.Next(&r)) {
      sum += (uint32_t)r.seq.size() + 1;
      if (sum > max_concat) {
        pending = r;
        pending_valid = true;
        sum -= (uint32_t)r.seq.size() + 1;
        break;
      }
      recs.push_back(r);
    }
    if (recs.empty()) {
      std::ofstream f((out_prefix + ".inf").c_str(), std::ios::binary);
      const int32_t division = chunk;
      WriteRaw(f, &division, 1);
      WriteRaw(f, &seed, 1);
      WriteRaw(f, &max_concat, 1);
      WriteRaw(f, &sum_length, 1);
      for (int k = 0; k < 32; ++k) WriteRaw(f, &division, 1);
      break;
    }
    const std::string prefix = out_prefix + "_" + std::to_string(chunk);
    // concatenation with END separators (X-filled, then overwritten)
    std::vector<uint32_t> starts(recs.size());
    uint32_t len = 0;
    for (size_t i = 0; i < recs.size(); ++i) {
      starts[i] = len;
      len += (uint32_t)recs[i].seq.size() + 1;
    }
    std::vector<uint8_t> data(len, kBaseX);
    for (size_t i = 0; i < recs.size(); ++i) {
      const std::string &s = recs[i].seq;
      for (size_t k = 0; k < s.size(); ++k) data[starts[i] + k] = ProteinCode((unsigned char)s[k]);
      data[starts[i] + s.size()] = kSeqEnd;
    }
    sum_length += len - recs.size();
    {
      std::ofstream f((prefix + ".inf").c_str(), std::ios::binary);
      const uint32_t n = (uint32_t)recs.size();
      WriteRaw(f, &n, 1);
      WriteRaw(f, &len, 1);
    }
    WriteNames(prefix + ".nam", recs);
    {
      std::ofstream f((prefix + ".seq").c_str(), std::ios::binary);
      WriteRaw(f, data.data(), data.size());
    }
    {
      std::ofstream f((prefix + ".pos").c_str(), std::ios::binary);
      WriteRaw(f, starts.data(), starts.size());
    }
    if (device >= 0) {
      std::vector<uint32_t> kc(kcl), pos(len);
      uint32_t npos = 0;
      if (GhostmBuildIndexGpu(data.data(), len, seed, kcl, kc.data(), pos.data(), &npos, device, nullptr))
        throw Error(std::string("db -D: ") + GhostmGetLastError());
      std::ofstream f((prefix + ".ind").c_str(), std::ios::binary);
      WriteRaw(f, &seed, 1);
      WriteRaw(f, &kcl, 1);
      WriteRaw(f, &npos, 1);
      WriteRaw(f, kc.data(), kc.size());
      WriteRaw(f, pos.data(), npos);
      continue;
    }
    // counting-sort k-mer index; windows containing X (anywhere in the seed span)
    // are skipped, subjects not longer than the seed span contribute nothing
    std::vector<uint32_t> key_at(len, UINT_MAX);
    std::vector<uint32_t> kc(kcl, 0);
    for (size_t i = 0; i < recs.size(); ++i) {
      if (recs[i].seq.size() <= seed_len) continue;
      for (uint32_t j = starts[i]; data[j + seed_len - 1] != kSeqEnd; ++j) {
        bool has_x = false;
        for (uint32_t t = 0; t < seed_len; ++t) has_x |= data[j + t] == kBaseX;
        if (has_x) continue;
        uint32_t key = 0, t = 0;
        for (uint32_t s = seed; s; s >>= 1, ++t)
          if (s & 1u) key = (key << kCharBits) | data[j + t];
        key_at[j] = key;
        ++kc[key + 1];
      }
    }
    for (uint32_t k = 1; k < kcl; ++k) kc[k] += kc[k - 1];
    const uint32_t npos = kc[kcl - 1];
    std::vector<uint32_t> pos(npos), fill(kcl, 0);
    for (size_t i = 0; i < recs.size(); ++i) {
      for (uint32_t j = starts[i]; data[j] != kSeqEnd; ++j) {
        const uint32_t key = key_at[j];
        if (key != UINT_MAX) pos[kc[key] + fill[key]++] = j;
      }
    }
    {
      std::ofstream f((prefix + ".ind").c_str(), std::ios::binary);
      WriteRaw(f, &seed, 1);
      WriteRaw(f, &kcl, 1);
      WriteRaw(f, &npos, 1);
      WriteRaw(f, kc.data(), kc.size());
      WriteRaw(f, pos.data(), pos.size());
    }
  }
  return 0;
}

// ------------------------------------------------------------------ qry
namespace {

// Standard genetic code indexed by 2-bit bases (A0 C1 G2 T3) first-base-major;
// entry 64 is any codon with an ambiguous base.
const char kCodons[] =
    "knkn" "tttt" "rsrs" "iimi"
    "qhqh" "pppp" "rrrr" "llll"
    "eded" "aaaa" "gggg" "vvvv"
    "*y*y" "ssss" "*cwc" "lflf"
    "x";

// Six reading frames of a read (forward 0..2, reverse complement 0..2). Stop
// codons switch the frame to '*' until the next ATG; frames are '*'-padded to
// dna_len/3 residues.
void SixFrames(const std::string &dna, uint32_t dna_len, std::vector<std::string> *frames) {
  std::vector<uint8_t> strand[2] = {std::vector<uint8_t>(dna_len), std::vector<uint8_t>(dna_len)};
  for (uint32_t j = 0; j < dna_len; ++j) {
    const uint8_t b = j < dna.size() ? DnaCode((unsigned char)dna[j]) : 4;
    strand[0][j] = b;
    strand[1][dna_len - j - 1] = b > 3 ? b : (uint8_t)((~b) & 3u);
  }
  const uint32_t width = dna_len / 3;
  frames->clear();
  for (int s = 0; s < 2; ++s) {
    for (uint32_t off = 0; off < 3; ++off) {
      std::string p;
      bool stop = false;
      for (uint32_t k = off + 2; k < dna_len; k += 3) {
        uint32_t codon = 0;
        for (int l = 2; l >= 0; --l) {
          const uint8_t b = strand[s][k - l];
          if (b > 3) { codon = 64; break; }
          codon = (codon << 2) | b;
        }
        if (codon == 14) stop = false;                              // ATG
        else if (codon == 48 || codon == 50 || codon == 56) stop = true;  // TAA TAG TGA
        p.push_back(stop ? '*' : kCodons[codon]);
      }
      while (p.size() < width) p.push_back('*');
      frames->push_back(p);
    }
  }
}

// qry -D: the chunk's letters concatenated, coded / translated on the GPU
// (qformat.hip), then the same files as the CPU path.
void FormatQueryChunkGpu(const std::vector<FastaRecord> &recs, bool dna, uint32_t width, int device,
                         const std::string &prefix) {
  const uint32_t n = (uint32_t)recs.size();
  std::vector<uint64_t> off(n);
  std::vector<uint32_t> len(n);
  uint64_t total = 0;
  for (uint32_t r = 0; r < n; ++r) {
    off[r] = total;
    len[r] = (uint32_t)recs[r].seq.size();
    total += len[r];
  }
  std::string raw;
  raw.reserve(total);
  for (const FastaRecord &r : recs) raw += r.seq;
  // every read is cut/padded to the first read's length (query_creator.cpp:254)
  const uint32_t dna_len = dna ? (uint32_t)recs[0].seq.size() : 0;
  const uint32_t per = dna ? 6 : 1;
  std::vector<uint8_t> out((size_t)n * per * width);
  if (GhostmFormatQueriesGpu(reinterpret_cast<const uint8_t *>(raw.data()), total, off.data(), len.data(), n,
                             width, dna ? std::max(dna_len, 1u) : 0, out.data(), device, nullptr))
    throw Error(std::string("qry -D: ") + GhostmGetLastError());
  {
    std::ofstream f((prefix + ".inf").c_str(), std::ios::binary);
    const uint32_t nout = n * per;
    WriteRaw(f, &nout, 1);
    WriteRaw(f, &width, 1);
  }
  {
    std::ofstream f((prefix + ".nam").c_str());
    for (const FastaRecord &r : recs)
      for (uint32_t k = 0; k < per; ++k) f << r.name << '\n';
  }
  // the CPU path's over-width warning, per record (frames: dna_len / 3 letters)
  for (const FastaRecord &r : recs) {
    const size_t letters = dna ? dna_len / 3 : r.seq.size();
    if (letters > width)
      for (uint32_t k = 0; k < per; ++k) std::cerr << "warning : the length of sequence is over. " << r.name << std::endl;
  }
  std::ofstream f((prefix + ".seq").c_str(), std::ios::binary);
  WriteRaw(f, out.data(), out.size());
}

}  // namespace

int QueryFormatMain(int argc, char **argv) {
  std::string in_path, out_prefix;
  uint32_t max_concat = 1u << 27;
  uint32_t width = 75;
  bool dna = false;
  int device = -1;  // -D d (extension): code / translate the records on GPU d
  optind = 1;
  int c;
  while ((c = getopt(argc, argv, "i:o:l:t:L:D:")) >= 0) {
    switch (c) {
      case 'i': in_path = optarg; break;
      case 'o': out_prefix = optarg; break;
      case 'l': width = atoi(optarg); break;
      case 'L': max_concat = atoi(optarg) * (1 << 20); break;
      case 'D': device = atoi(optarg); break;
      case 't':
        if (strcmp(optarg, "d") == 0) dna = true;
        else if (strcmp(optarg, "p") == 0) dna = false;
        else throw std::invalid_argument("-t is not support " + std::string(optarg) + ".");
        break;
      default: throw std::invalid_argument("");
    }
  }
  if (dna) {
    max_concat /= 2;
    width /= 3;
    if (width >= kMaxQueryLength) {
      std::cerr << "Warring: over upper limit of query length. Max is " << kMaxQueryLength * 3 << "." << std::endl;
      width = kMaxQueryLength;
    }
  } else if (width >= kMaxQueryLength) {
    std::cerr << "Warring: over upper limit of query length. Max is " << kMaxQueryLength << "." << std::endl;
    width = kMaxQueryLength;
  }
  FastaReader reader(in_path);
  bool pending_valid = false;
  FastaRecord pending;
  uint32_t max_nseq = 0;
  for (int chunk = 0;; ++chunk) {
    std::vector<FastaRecord> recs;
    uint32_t sum = 0;
    if (pending_valid) {
      sum = (uint32_t)pending.seq.size();
      if (sum > max_concat) {
        std::cerr << "error : too small max length." << std::endl;
        return 1;
      }
      recs.push_back(pending);
      pending_valid = false;
    }
    FastaRecord r;
    while (reader.Next(&r)) {
      sum += (uint32_t)r.seq.size();
      if (sum > max_concat) {
        pending = r;
        pending_valid = true;
        break;
      }
      recs.push_back(r);
    }
    if (recs.empty()) {
      std::ofstream f((out_prefix + ".inf").c_str(), std::ios::binary);
      const int32_t division = chunk;
      WriteRaw(f, &division, 1);
      WriteRaw(f, &width, 1);
      WriteRaw(f, &max_nseq, 1);
      for (int k = 0; k < 32; ++k) WriteRaw(f, &division, 1);
      break;
    }
    if (device >= 0) {
      FormatQueryChunkGpu(recs, dna, width, device, out_prefix + "_" + std::to_string(chunk));
      const uint32_t nout = (uint32_t)recs.size() * (dna ? 6u : 1u);
      if (max_nseq < nout) max_nseq = nout;
      continue;
    }
    if (dna) {
      // every read is cut/padded to the first read's length (query_creator.cpp:254)
      const uint32_t dna_len = (uint32_t)recs[0].seq.size();
      std::vector<FastaRecord> prot;
      std::vector<std::string> frames;
      for (const FastaRecord &d : recs) {
        SixFrames(d.seq, dna_len, &frames);
        for (std::string &f : frames) prot.push_back(FastaRecord{d.name, f});
      }
      recs.swap(prot);
    }
    if (max_nseq < recs.size()) max_nseq = (uint32_t)recs.size();
    const std::string prefix = out_prefix + "_" + std::to_string(chunk);
    {
      std::ofstream f((prefix + ".inf").c_str(), std::ios::binary);
      const uint32_t n = (uint32_t)recs.size();
      WriteRaw(f, &n, 1);
      WriteRaw(f, &width, 1);
    }
    WriteNames(prefix + ".nam", recs);
    std::ofstream f((prefix + ".seq").c_str(), std::ios::binary);
    std::vector<uint8_t> rec(width);
    for (const FastaRecord &q : recs) {
      size_t n = q.seq.size();
      if (n > width) {
        std::cerr << "warning : the length of sequence is over. " << q.name << std::endl;
        n = width;
      }
      for (size_t k = 0; k < n; ++k) rec[k] = ProteinCode((unsigned char)q.seq[k]);
      for (size_t k = n; k < width; ++k) rec[k] = kBaseX;
      WriteRaw(f, rec.data(), width);
    }
  }
  return 0;
}

}  // namespace ghostm
