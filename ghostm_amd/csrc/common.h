// common.h — constants of the GHOSTM data model (reference common.h:29-44) and
// small host helpers shared by the native library.
#pragma once
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

namespace ghostm {

constexpr int kAlphabet = 32;        // codes per residue slot (5 bits)
constexpr int kCharBits = 5;         // bits per residue in a k-mer key
constexpr uint8_t kSeqEnd = 25;      // subject separator in the concatenated DB
constexpr uint8_t kBaseX = 23;       // unknown residue / query padding
constexpr uint32_t kMaxQueryLength = 127;  // MAX_COLUMN_LENGTH - 1

// Protein letter -> code (reference sequence.cpp:63-87): A R N D C Q E G H I L K
// M F P S T W Y V B J Z X * get 0..24, both cases; every other byte is X.
uint8_t ProteinCode(unsigned char ch);
// DNA letter -> code (sequence.cpp:34-59): A0 C1 G2 T3, '-' 5, other 4.
uint8_t DnaCode(unsigned char ch);

struct Error : std::runtime_error {
  explicit Error(const std::string &m) : std::runtime_error(m) {}
};

inline double NowSeconds() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

// GHOSTM_TRACE=1: a host timeline of each GhostmSessionRun (label, value,
// thread, ms since the run started), printed to stderr when the run ends.
bool TraceOn();
double ThreadCpuSeconds();  // this thread's CPU time (CLOCK_THREAD_CPUTIME_ID)
void TraceMark(const char *label, uint64_t value = 0);
void TraceDump();

}  // namespace ghostm
