// capi.cpp — session part of the C ABI (include/ghostm_hip.h Part 2).
#include <algorithm>
#include <cstring>
#include <fstream>
#include <iostream>
#include <vector>

#include "../../include/ghostm_hip.h"
#include "aligner.h"
#include "common.h"

using namespace ghostm;

namespace ghostm {
void SetLastErrorMessage(const std::string &m);
}

extern "C" {

void *GhostmSessionCreate(int argc, char **argv) {
  try {
    AlignerOptions opt = ParseAlignerOptions(argc, argv);
    return new Session(opt);
  } catch (std::exception &e) {
    SetLastErrorMessage(e.what());
    return nullptr;
  }
}

void *GhostmSessionCreateShardEx(int argc, char **argv, int rank, int world, GhostmAllGatherFn allgather,
                                 void *ctx) {
  try {
    if (world < 1 || rank < 0 || rank >= world) throw Error("shard rank outside 0..world-1");
    AlignerOptions opt = ParseAlignerOptions(argc, argv);
    ShardExchange ex;
    ex.fn = allgather;
    ex.ctx = ctx;
    return new Session(opt, (uint32_t)rank, (uint32_t)world, &ex);
  } catch (std::exception &e) {
    SetLastErrorMessage(e.what());
    return nullptr;
  }
}

void *GhostmSessionCreateShard(int argc, char **argv, int rank, int world) {
  return GhostmSessionCreateShardEx(argc, argv, rank, world, nullptr, nullptr);
}

int GhostmSessionShardRange(void *s, uint64_t *begin, uint64_t *end) {
  if (!s) return 1;
  const Session *p = static_cast<Session *>(s);
  if (begin) *begin = p->ShardBegin();
  if (end) *end = p->ShardEnd();
  return 0;
}

uint64_t GhostmSessionHitCapacity(void *s) {
  if (!s) return UINT64_MAX;
  return static_cast<Session *>(s)->HitCapacity();
}

int GhostmShardCuts(uint64_t n, const uint32_t weights[], const uint8_t group_start[], int world,
                    uint64_t cuts[]) {
  try {
    if (world < 1) throw Error("world must be >= 1");
    ShardCuts(n, weights, group_start, (uint32_t)world, cuts);
    return 0;
  } catch (std::exception &e) {
    SetLastErrorMessage(e.what());
    return 1;
  }
}

int GhostmSessionRun(void *s) {
  try {
    if (!s) throw Error("null session");
    static_cast<Session *>(s)->Run();
    return 0;
  } catch (std::exception &e) {
    SetLastErrorMessage(e.what());
    return 1;
  }
}

int GhostmSessionRunToFile(void *s) {
  try {
    if (!s) throw Error("null session");
    static_cast<Session *>(s)->Run(true);
    return 0;
  } catch (std::exception &e) {
    SetLastErrorMessage(e.what());
    return 1;
  }
}

size_t GhostmSessionOutput(void *s, char *buf, size_t cap) {
  if (!s) return 0;
  const std::string &o = static_cast<Session *>(s)->Output();
  if (!buf) return o.size();
  const size_t n = std::min(cap, o.size());
  std::memcpy(buf, o.data(), n);
  return n;
}

int GhostmSessionWrite(void *s) {
  try {
    if (!s) throw Error("null session");
    static_cast<Session *>(s)->WriteOutputFile();
    return 0;
  } catch (std::exception &e) {
    SetLastErrorMessage(e.what());
    return 1;
  }
}

size_t GhostmSessionHits(void *s, GhostmHit *hits, size_t cap) {
  if (!s) return 0;
  const std::vector<GhostmHit> &h = static_cast<Session *>(s)->Hits();
  if (!hits) return h.size();
  const size_t n = std::min(cap, h.size());
  std::memcpy(hits, h.data(), n * sizeof(GhostmHit));
  return n;
}

size_t GhostmSessionDeviceHits(void *s, void *dst_device, size_t cap) {
  try {
    if (!s) throw Error("null session");
    return static_cast<Session *>(s)->DeviceHits(dst_device, cap);
  } catch (std::exception &e) {
    SetLastErrorMessage(e.what());
    return (size_t)-1;
  }
}

int GhostmSessionStats(void *s, GhostmStats *stats) {
  if (!s || !stats) return 1;
  *stats = static_cast<Session *>(s)->Stats();
  return 0;
}

size_t GhostmSessionStatsSized(void *s, GhostmStats *stats, size_t size) {
  if (!s || !stats) return 0;
  const GhostmStats &st = static_cast<Session *>(s)->Stats();
  std::memcpy(stats, &st, std::min(size, sizeof(GhostmStats)));
  return sizeof(GhostmStats);
}

void GhostmSessionDestroy(void *s) { delete static_cast<Session *>(s); }

// `ghostm aln` (reference Aligner::Execute via main.cpp:107-121): the output file
// is opened right after option parsing; every error is printed and 0 returned.
int GhostmAlignMain(int argc, char **argv) {
  try {
    AlignerOptions opt = ParseAlignerOptions(argc, argv);
    { std::ofstream touch(opt.output_file.c_str()); }
    Session session(opt);
    session.Run(true);       // the output file is written while the search runs
    session.WriteOutputFile();  // no-op after a streamed run
    if (opt.verbose) {
      const GhostmStats &st = session.Stats();
      std::cout << "# queries " << st.queries << " candidates " << st.candidates << " hits "
                << st.hits << "\n# seconds total " << st.seconds_total << " seed " << st.seconds_seed
                << " score " << st.seconds_score << " traceback " << st.seconds_traceback
                << " merge " << st.seconds_merge << " output " << st.seconds_output << std::endl;
    }
  } catch (std::exception &e) {
    std::cerr << e.what() << std::endl;
  }
  return 0;
}

}  // extern "C"
