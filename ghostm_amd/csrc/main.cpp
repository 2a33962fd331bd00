// main.cpp — the `ghostm` command line (reference main.cpp:36-122): db | qry | aln,
// plus `synth` (synthetic benchmark inputs). `aln` always runs on the GPU
// (-D selects the device, default 0). Errors are printed and the process exits 0
// like the reference; usage or an unknown command exits 1.
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <stdexcept>

#include "../../include/ghostm_hip.h"

namespace ghostm {
int DbFormatMain(int argc, char **argv);
int QueryFormatMain(int argc, char **argv);
int SynthMain(int argc, char **argv);
}  // namespace ghostm

static int Usage() {
  std::cerr << "ghostm (MI355X build of GHOSTM 2.0)\n"
            << "Command and Options\n"
            << "db:  ghostm db [-i dbFastaFile] [-o dbName] [-k kSize] [-l chunkSize]\n"
            << "qry: ghostm qry [-i qryFastaFile] [-o qryName] [-l maxLength] [-L chunkSize] [-t d|p]\n"
            << "aln: ghostm aln [-b best] [-D deviceId] [-l CandidatesSize] [-s skipSize]\n"
            << "       [-t threshold] [-r regionSize] [-e extendSize] [-G openGap] [-E extendGap]\n"
            << "       [-M scoreMatrix] [-y outputStyle] [-S startChunk] [-L endChunk] [-v]\n"
            << "       -i queries -d database -o output\n"
            << "synth: ghostm synth -d db.fasta -q queries.fasta [-n nq] [-N dbResidues] [-s seed]\n";
  return 1;
}

int main(int argc, char **argv) {
  if (argc < 2) return Usage();
  const char *cmd = argv[1];
  try {
    if (strcmp(cmd, "aln") == 0) {
      const int rc = GhostmAlignMain(argc - 1, argv + 1);
      // the session is gone and its output file closed: leave without the HIP
      // runtime's teardown (tens of ms of a cold run; GHOSTM_FAST_EXIT=0 keeps it)
      std::cout.flush();
      std::cerr.flush();
      std::fflush(nullptr);
      const char *e = std::getenv("GHOSTM_FAST_EXIT");
      if (!(e && std::strcmp(e, "0") == 0)) _exit(rc);
      return rc;
    }
    if (strcmp(cmd, "db") == 0) { ghostm::DbFormatMain(argc - 1, argv + 1); return 0; }
    if (strcmp(cmd, "qry") == 0) { ghostm::QueryFormatMain(argc - 1, argv + 1); return 0; }
    if (strcmp(cmd, "synth") == 0) return ghostm::SynthMain(argc - 1, argv + 1);
  } catch (std::exception &e) {
    std::cerr << e.what() << std::endl;
    return 0;
  }
  std::cerr << "[main] unrecognized command " << cmd << std::endl;
  return 1;
}
