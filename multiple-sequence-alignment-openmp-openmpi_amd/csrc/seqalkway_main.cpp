// seqalkway_main.cpp -- the host driver with the reference's stdin/stdout
// contract (seqalign-mpi-skeleton.cpp:35-76, "do not change" above :78).
//
//   stdin : pxy pgap k seq_0 ... seq_{k-1}   (whitespace-separated tokens)
//   stdout: "Time: <us> us" / answer hash / penalties each followed by ' '
//
// Extensions (stdout unchanged):
//   --fasta FILE --pxy P --pgap G   sequences from a FASTA file instead of stdin
//                                   (records in file order; header lines start
//                                   with '>', sequence lines concatenated with
//                                   whitespace removed)
//   --dump FILE                     per pair in canonical order: "i j penalty",
//                                   then align1 and align2 (trimmed rows) lines
//   --print-inputs                  parse only (no GPU): k, then "<length> <sha512>"
//                                   per sequence -- the parser parity hook
//   --msa FILE                      progressive sum-of-pairs MSA (SURVEY §8 f3,
//                                   nwk_msa) as FASTA: ">seq<i> sop=<score>"
//                                   headers, one aligned row per record
//
// The timed span is the getMinimumPenalties call (skel:53-61), here
// nwk_get_minimum_penalties.  No MPI: the reference's ranks become devices
// (--gpus N or NWK_GPUS=N); flags and statistics never change stdout.
#include <sys/time.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "../../include/nwk.h"

static uint64_t GetTimeStamp() {
  struct timeval tv;
  gettimeofday(&tv, NULL);
  return tv.tv_sec * (uint64_t)1000000 + tv.tv_usec;
}

// FASTA records in file order (see header).
static bool read_fasta(const char* path, std::vector<std::string>* out) {
  std::ifstream in(path, std::ios::binary);
  if (!in) return false;
  std::string line;
  bool any = false;
  while (std::getline(in, line)) {
    if (!line.empty() && line[0] == '>') {
      out->emplace_back();
      any = true;
      continue;
    }
    bool blank = true;  // whitespace-only lines ("\r" of a CRLF blank line too) are skipped,
    for (char ch : line)  // as seqalign.parse_fasta's `not line.strip()`
      if (!isspace((unsigned char)ch)) { blank = false; break; }
    if (blank || line[0] == ';') continue;
    if (!any) {  // sequence text before the first header: an unnamed record
      out->emplace_back();
      any = true;
    }
    for (char ch : line)
      if (!isspace((unsigned char)ch)) out->back().push_back(ch);
  }
  return true;
}

// Rows of every pair (one device, single-pair entry point) into `path`.
static int dump_pairs(const char* path, const std::vector<std::string>& genes, int pxy, int pgap) {
  FILE* f = fopen(path, "w");
  if (!f) return NWK_EINVAL;
  nwk_ctx* ctx = nullptr;
  int rc = nwk_ctx_create(nullptr, &ctx);
  for (size_t i = 1; rc == NWK_OK && i < genes.size(); ++i)
    for (size_t j = 0; rc == NWK_OK && j < i; ++j) {
      const std::string &x = genes[i], &y = genes[j];
      std::vector<uint8_t> a1(x.size() + y.size() + 1), a2(x.size() + y.size() + 1);
      int32_t alen = 0, pen = 0;
      rc = nwk_get_minimum_penalty(ctx, reinterpret_cast<const uint8_t*>(x.data()), (int32_t)x.size(),
                                   reinterpret_cast<const uint8_t*>(y.data()), (int32_t)y.size(), pxy, pgap,
                                   a1.data(), a2.data(), &alen, &pen);
      if (rc == NWK_OK)
        fprintf(f, "%zu %zu %d\n%.*s\n%.*s\n", i, j, pen, alen, (const char*)a1.data(), alen, (const char*)a2.data());
    }
  nwk_ctx_destroy(ctx);
  fclose(f);
  return rc;
}

// Progressive SoP MSA of `genes` from the call's pairwise penalties into `path` (FASTA).
static int write_msa(const char* path, const std::vector<std::string>& genes, const std::string& all,
                     const std::vector<int64_t>& off, int pxy, int pgap, const std::vector<int32_t>& penalties) {
  FILE* f = fopen(path, "w");
  if (!f) return NWK_EINVAL;
  nwk_ctx* ctx = nullptr;
  int rc = nwk_ctx_create(nullptr, &ctx);
  const int64_t cap = off.back() > 0 ? off.back() : 1;
  std::vector<uint8_t> rows((size_t)cap * (genes.empty() ? 1 : genes.size()));
  int64_t len = 0, sop = 0;
  if (rc == NWK_OK)
    rc = nwk_set_sequences(ctx, reinterpret_cast<const uint8_t*>(all.data()), off.data(), (int32_t)genes.size());
  if (rc == NWK_OK) rc = nwk_msa(ctx, pxy, pgap, penalties.data(), rows.data(), cap, &len, &sop);
  for (size_t r = 0; rc == NWK_OK && r < genes.size(); ++r)
    fprintf(f, ">seq%zu sop=%lld\n%.*s\n", r, (long long)sop, (int)len, (const char*)rows.data() + r * cap);
  nwk_ctx_destroy(ctx);
  fclose(f);
  return rc;
}

int main(int argc, char** argv) {
  nwk_opts o;
  nwk_opts_default(&o);
  if (const char* g = getenv("NWK_GPUS")) o.ngpus = atoi(g);
  if (const char* v = getenv("NWK_VERBOSE")) o.verbose = atoi(v);
  if (const char* b = getenv("NWK_BITS")) o.bits = atoi(b);
  const char *fasta = nullptr, *dump = nullptr, *msa = nullptr;
  bool print_inputs = false;
  int fpxy = 3, fpgap = 2;
  for (int a = 1; a < argc; ++a) {
    if (!strcmp(argv[a], "--gpus") && a + 1 < argc) o.ngpus = atoi(argv[++a]);
    else if (!strcmp(argv[a], "--verbose")) o.verbose = 1;
    else if (!strcmp(argv[a], "--bits") && a + 1 < argc) o.bits = atoi(argv[++a]);
    else if (!strcmp(argv[a], "--fasta") && a + 1 < argc) fasta = argv[++a];
    else if (!strcmp(argv[a], "--pxy") && a + 1 < argc) fpxy = atoi(argv[++a]);
    else if (!strcmp(argv[a], "--pgap") && a + 1 < argc) fpgap = atoi(argv[++a]);
    else if (!strcmp(argv[a], "--dump") && a + 1 < argc) dump = argv[++a];
    else if (!strcmp(argv[a], "--msa") && a + 1 < argc) msa = argv[++a];
    else if (!strcmp(argv[a], "--print-inputs")) print_inputs = true;
    else {
      fprintf(stderr,
              "usage: %s [--gpus N] [--bits W] [--verbose] [--fasta FILE --pxy P --pgap G] [--dump FILE] [--msa FILE] [--print-inputs] [< input]\n",
              argv[0]);
      return 2;
    }
  }
  std::ios::sync_with_stdio(false);
  int misMatchPenalty = 0, gapPenalty = 0, k = 0;
  std::vector<std::string> genes;
  if (fasta) {
    if (!read_fasta(fasta, &genes)) {
      fprintf(stderr, "seqalkway: cannot read %s\n", fasta);
      return 1;
    }
    misMatchPenalty = fpxy;
    gapPenalty = fpgap;
    k = (int)genes.size();
  } else {
    std::cin >> misMatchPenalty >> gapPenalty >> k;
    if (k < 0) k = 0;
    genes.resize((size_t)k);
    for (int i = 0; i < k; i++) std::cin >> genes[i];
  }
  if (print_inputs) {
    printf("%d\n", k);
    for (auto& g : genes) {
      char hx[NWK_HASH_HEX];
      nwk_sha512_hex(reinterpret_cast<const uint8_t*>(g.data()), (int64_t)g.size(), hx);
      printf("%zu %s\n", g.size(), hx);
    }
    return 0;
  }
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
  if (dump && (rc = dump_pairs(dump, genes, misMatchPenalty, gapPenalty)) != NWK_OK) {
    fprintf(stderr, "seqalkway: --dump: error %d: %s\n", rc, nwk_last_error());
    return 1;
  }
  if (msa && (rc = write_msa(msa, genes, all, off, misMatchPenalty, gapPenalty, penalties)) != NWK_OK) {
    fprintf(stderr, "seqalkway: --msa: error %d: %s\n", rc, nwk_last_error());
    return 1;
  }
  return 0;
}
