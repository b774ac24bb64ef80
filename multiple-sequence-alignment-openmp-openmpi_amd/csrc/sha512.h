// sha512.h -- FIPS 180-4 SHA-512 for the host side of the engine.
//
// Replaces sw::sha512 (reference sha512.hh:59-296).  The reference writes only
// the low 32 bits of the message bit length (sha512.hh:131,141); for every
// message shorter than 2^29 bytes that equals the standard encoding used
// here, and alignment rows are at most 2*100k bytes (Project2B.pdf p.5).
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace nwk {

struct Sha512 {
  uint64_t st[8];
  uint64_t total;
  unsigned char buf[128];
  size_t fill;

  Sha512() { reset(); }
  void reset();
  void update(const void* data, size_t len);
  void final(unsigned char out[64]);
};

void sha512_raw(const void* data, size_t len, unsigned char out[64]);
// 128 lowercase hex chars, no terminator.
void to_hex(const unsigned char raw[64], char hex[128]);
void sha512_hex(const void* data, size_t len, char hex[128]);

// The answer-hash chain of skel:159, acc <- sha512hex(acc ++ hex(problemhash)),
// link by link.  Its message is 128 hex chars of acc, 128 of the problem hash
// and a constant padding block, so per link only the first block's schedule
// depends on acc: the second block's K + W (chain_schedule, any thread, ahead
// of the chain) and the padding block's are precomputed, and acc stays binary
// (hex digits are formed in registers).  chain_step is bit-identical to
// sha512_hex on the concatenation.
struct ChainAcc {
  uint64_t dig[8];
  bool empty = true;  // acc == "" (skel:121)
};
void chain_schedule(const unsigned char problem_hash[64], uint64_t kw[80]);
void chain_step(ChainAcc* acc, const uint64_t kw[80]);
void chain_hex(const ChainAcc& acc, char hex[128]);  // (empty acc: nothing to write)

}  // namespace nwk
