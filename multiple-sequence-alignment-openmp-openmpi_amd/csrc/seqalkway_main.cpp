// seqalkway_main.cpp -- the host driver with the reference's stdin/stdout
// contract (seqalign-mpi-skeleton.cpp:35-76, "do not change" above :78).
//
//   stdin : pxy pgap k seq_0 ... seq_{k-1}   (whitespace-separated tokens)
//   stdout: "Time: <us> us" / answer hash / penalties each followed by ' '
//
// The timed span is the getMinimumPenalties call (skel:53-61), here
// nwk_get_minimum_penalties.  No MPI: the reference's ranks become devices
// (--gpus N or NWK_GPUS=N); flags and statistics never change stdout.
#include <sys/time.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "../../include/nwk.h"

static uint64_t GetTimeStamp() {
  struct timeval tv;
  gettimeofday(&tv, NULL);
  return tv.tv_sec * (uint64_t)1000000 + tv.tv_usec;
}

int main(int argc, char** argv) {
  nwk_opts o;
  nwk_opts_default(&o);
  if (const char* g = getenv("NWK_GPUS")) o.ngpus = atoi(g);
  if (const char* v = getenv("NWK_VERBOSE")) o.verbose = atoi(v);
  if (const char* b = getenv("NWK_BITS")) o.bits = atoi(b);
  for (int a = 1; a < argc; ++a) {
    if (!strcmp(argv[a], "--gpus") && a + 1 < argc) o.ngpus = atoi(argv[++a]);
    else if (!strcmp(argv[a], "--verbose")) o.verbose = 1;
    else if (!strcmp(argv[a], "--bits") && a + 1 < argc) o.bits = atoi(argv[++a]);
    else {
      fprintf(stderr, "usage: %s [--gpus N] [--bits W] [--verbose] < input\n", argv[0]);
      return 2;
    }
  }
  std::ios::sync_with_stdio(false);
  int misMatchPenalty = 0, gapPenalty = 0, k = 0;
  std::cin >> misMatchPenalty >> gapPenalty >> k;
  if (k < 0) k = 0;
  std::vector<std::string> genes((size_t)k);
  for (int i = 0; i < k; i++) std::cin >> genes[i];
  std::vector<int64_t> off((size_t)k + 1, 0);
  for (int i = 0; i < k; i++) off[i + 1] = off[i] + (int64_t)genes[i].size();
  std::string all;
  all.reserve((size_t)off[k]);
  for (auto& g : genes) all += g;
  const int64_t numPairs = (int64_t)k * (k - 1) / 2;
  std::vector<int32_t> penalties((size_t)(numPairs > 0 ? numPairs : 1));
  char hash[NWK_HASH_HEX];

  uint64_t start = GetTimeStamp();
  int rc = nwk_get_minimum_penalties(reinterpret_cast<const uint8_t*>(all.data()), off.data(), k,
                                     misMatchPenalty, gapPenalty, penalties.data(), hash, &o);
  uint64_t el = GetTimeStamp() - start;
  if (rc != NWK_OK) {
    fprintf(stderr, "seqalkway: error %d: %s\n", rc, nwk_last_error());
    return 1;
  }
  printf("Time: %ld us\n", (long)el);
  fflush(stdout);
  std::cout << hash << std::endl;
  for (int64_t i = 0; i < numPairs; i++) std::cout << penalties[i] << " ";
  std::cout << std::endl;
  return 0;
}
