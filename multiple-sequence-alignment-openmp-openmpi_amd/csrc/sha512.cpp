// sha512.cpp -- FIPS 180-4 SHA-512 (see sha512.h).
#include "sha512.h"

#include <string.h>

namespace nwk {

namespace {

constexpr uint64_t kK[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

inline uint64_t rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

inline uint64_t load_be64(const unsigned char* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return __builtin_bswap64(v);
}

// Fully unrolled rounds over a rolling 16-word message schedule; the eight
// working variables rotate by renaming (no moves), so each round is the
// FIPS 180-4 arithmetic and nothing else.
#define NWK_S0(x) (rotr(x, 28) ^ rotr(x, 34) ^ rotr(x, 39))
#define NWK_S1(x) (rotr(x, 14) ^ rotr(x, 18) ^ rotr(x, 41))
#define NWK_s0(x) (rotr(x, 1) ^ rotr(x, 8) ^ ((x) >> 7))
#define NWK_s1(x) (rotr(x, 19) ^ rotr(x, 61) ^ ((x) >> 6))
#define NWK_ROUND(a, b, c, d, e, f, g, h, t, wt)                                   \
  do {                                                                          \
    const uint64_t t1 = h + NWK_S1(e) + (g ^ (e & (f ^ g))) + kK[t] + (wt);      \
    const uint64_t t2 = NWK_S0(a) + ((a & b) | (c & (a | b)));                  \
    d += t1;                                                                    \
    h = t1 + t2;                                                                \
  } while (0)

void compress(uint64_t st[8], const unsigned char* blk) {
  uint64_t w[16];
  for (int t = 0; t < 16; ++t) w[t] = load_be64(blk + 8 * t);
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int t = 0; t < 80; t += 8) {
    if (t >= 16) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int u = t + q;
        w[u & 15] += NWK_s1(w[(u - 2) & 15]) + w[(u - 7) & 15] + NWK_s0(w[(u - 15) & 15]);
      }
    }
    NWK_ROUND(a, b, c, d, e, f, g, h, t + 0, w[(t + 0) & 15]);
    NWK_ROUND(h, a, b, c, d, e, f, g, t + 1, w[(t + 1) & 15]);
    NWK_ROUND(g, h, a, b, c, d, e, f, t + 2, w[(t + 2) & 15]);
    NWK_ROUND(f, g, h, a, b, c, d, e, t + 3, w[(t + 3) & 15]);
    NWK_ROUND(e, f, g, h, a, b, c, d, t + 4, w[(t + 4) & 15]);
    NWK_ROUND(d, e, f, g, h, a, b, c, t + 5, w[(t + 5) & 15]);
    NWK_ROUND(c, d, e, f, g, h, a, b, t + 6, w[(t + 6) & 15]);
    NWK_ROUND(b, c, d, e, f, g, h, a, t + 7, w[(t + 7) & 15]);
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
  st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}
// The chain's rounds (latency-bound: one dependent compression after another).
// Maj(a, b, c) = b ^ ((a ^ b) & (b ^ c)) with (b ^ c) carried over from the
// previous round's (a ^ b), and h + K + W summed off the e / a critical paths:
// 354 vs 400 ns per chain link on the MI355X box's EPYC 9575F
// (tools/probe/chain_probe2.cpp).
#define NWK_RC(a, b, c, d, e, f, g, h, kw, AB, BC)                      \
  do {                                                                \
    const uint64_t t1 = (h + (kw)) + (g ^ (e & (f ^ g))) + NWK_S1(e); \
    AB = a ^ b;                                                       \
    d += t1;                                                          \
    h = t1 + (NWK_S0(a) + (b ^ (AB & BC)));                           \
  } while (0)

// Compression over a precomputed K + W schedule (the chain's fixed blocks).
void compress_kw(uint64_t st[8], const uint64_t kw[80]) {
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  uint64_t x = b ^ c, y;
#pragma unroll
  for (int t = 0; t < 80; t += 8) {
    NWK_RC(a, b, c, d, e, f, g, h, kw[t + 0], y, x);
    NWK_RC(h, a, b, c, d, e, f, g, kw[t + 1], x, y);
    NWK_RC(g, h, a, b, c, d, e, f, kw[t + 2], y, x);
    NWK_RC(f, g, h, a, b, c, d, e, kw[t + 3], x, y);
    NWK_RC(e, f, g, h, a, b, c, d, kw[t + 4], y, x);
    NWK_RC(d, e, f, g, h, a, b, c, kw[t + 5], x, y);
    NWK_RC(c, d, e, f, g, h, a, b, kw[t + 6], y, x);
    NWK_RC(b, c, d, e, f, g, h, a, kw[t + 7], x, y);
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
  st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// Compression of a block given as 16 big-endian words, its schedule rolled
// into the rounds (the chain's first block, hex(acc): no schedule pass ahead
// of the rounds on the link's critical path)
void compress_w16(uint64_t st[8], uint64_t w[16]) {
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  uint64_t x = b ^ c, y;
#pragma unroll
  for (int t = 0; t < 80; t += 8) {
    if (t >= 16) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int u = t + q;
        w[u & 15] += NWK_s1(w[(u - 2) & 15]) + w[(u - 7) & 15] + NWK_s0(w[(u - 15) & 15]);
      }
    }
    NWK_RC(a, b, c, d, e, f, g, h, kK[t + 0] + w[(t + 0) & 15], y, x);
    NWK_RC(h, a, b, c, d, e, f, g, kK[t + 1] + w[(t + 1) & 15], x, y);
    NWK_RC(g, h, a, b, c, d, e, f, kK[t + 2] + w[(t + 2) & 15], y, x);
    NWK_RC(f, g, h, a, b, c, d, e, kK[t + 3] + w[(t + 3) & 15], x, y);
    NWK_RC(e, f, g, h, a, b, c, d, kK[t + 4] + w[(t + 4) & 15], y, x);
    NWK_RC(d, e, f, g, h, a, b, c, kK[t + 5] + w[(t + 5) & 15], x, y);
    NWK_RC(c, d, e, f, g, h, a, b, kK[t + 6] + w[(t + 6) & 15], y, x);
    NWK_RC(b, c, d, e, f, g, h, a, kK[t + 7] + w[(t + 7) & 15], x, y);
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
  st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}
#undef NWK_RC

// K + W of a block given as 16 big-endian words
void schedule_kw(const uint64_t w16[16], uint64_t kw[80]) {
  uint64_t w[80];
  for (int t = 0; t < 16; ++t) w[t] = w16[t];
  for (int t = 16; t < 80; ++t) w[t] = NWK_s1(w[t - 2]) + w[t - 7] + NWK_s0(w[t - 15]) + w[t - 16];
  for (int t = 0; t < 80; ++t) kw[t] = kK[t] + w[t];
}

#undef NWK_ROUND
#undef NWK_S0
#undef NWK_S1
#undef NWK_s0
#undef NWK_s1

// The 8 lowercase hex digits of the low 32 bits of x, most significant first,
// as one big-endian message word (SWAR: nibbles spread to bytes, +'0', +39
// more for a..f).
inline uint64_t hex_word(uint64_t x) {
  x &= 0xffffffffULL;
  x = (x | (x << 16)) & 0x0000FFFF0000FFFFULL;
  x = (x | (x << 8)) & 0x00FF00FF00FF00FFULL;
  x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0FULL;
  const uint64_t gt9 = ((x + 0x0606060606060606ULL) >> 4) & 0x0101010101010101ULL;
  return x + 0x3030303030303030ULL + gt9 * 0x27;
}

// the hex block of a 64-byte digest given as 8 big-endian words
inline void hex_block(const uint64_t d[8], uint64_t w16[16]) {
  for (int q = 0; q < 8; ++q) {
    w16[2 * q] = hex_word(d[q] >> 32);
    w16[2 * q + 1] = hex_word(d[q]);
  }
}

const uint64_t kIV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                         0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                         0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

// padding blocks of 128- and 256-byte messages: 0x80, zeros, the bit length
struct PadKW {
  uint64_t kw128[80], kw256[80];
  PadKW() {
    uint64_t w[16] = {0x8000000000000000ULL};
    w[15] = 128 * 8;
    schedule_kw(w, kw128);
    w[15] = 256 * 8;
    schedule_kw(w, kw256);
  }
};
const PadKW& pad_kw() {
  static const PadKW p;
  return p;
}

}  // namespace

void chain_schedule(const unsigned char ph[64], uint64_t kw[80]) {
  uint64_t d[8], w16[16];
  for (int q = 0; q < 8; ++q) d[q] = load_be64(ph + 8 * q);
  hex_block(d, w16);
  schedule_kw(w16, kw);
}

void chain_step(ChainAcc* acc, const uint64_t kw[80]) {
  uint64_t st[8];
  memcpy(st, kIV, sizeof st);
  if (acc->empty) {  // message = hex(ph): its block, then the padding of a 128-byte message
    compress_kw(st, kw);
    compress_kw(st, pad_kw().kw128);
    acc->empty = false;
  } else {           // message = hex(acc) ++ hex(ph), then the padding of a 256-byte message
    uint64_t w16[16];
    hex_block(acc->dig, w16);
    compress_w16(st, w16);
    compress_kw(st, kw);
    compress_kw(st, pad_kw().kw256);
  }
  memcpy(acc->dig, st, sizeof st);
}

void chain_hex(const ChainAcc& acc, char hex[128]) {
  if (acc.empty) return;
  unsigned char raw[64];
  for (int i = 0; i < 8; ++i) {
    const uint64_t v = __builtin_bswap64(acc.dig[i]);
    memcpy(raw + 8 * i, &v, 8);
  }
  to_hex(raw, hex);
}

void Sha512::reset() {
  static const uint64_t iv[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                 0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  memcpy(st, iv, sizeof st);
  total = 0;
  fill = 0;
}

void Sha512::update(const void* data, size_t len) {
  const unsigned char* p = static_cast<const unsigned char*>(data);
  total += len;
  if (fill) {
    const size_t take = len < 128 - fill ? len : 128 - fill;
    memcpy(buf + fill, p, take);
    fill += take; p += take; len -= take;
    if (fill < 128) return;
    compress(st, buf);
    fill = 0;
  }
  while (len >= 128) { compress(st, p); p += 128; len -= 128; }
  if (len) { memcpy(buf, p, len); fill = len; }
}

void Sha512::final(unsigned char out[64]) {
  const uint64_t bits = total * 8u;
  unsigned char pad[256] = {0x80};
  const size_t padlen = (fill < 112 ? 112 - fill : 240 - fill);
  update(pad, padlen);
  unsigned char lenbuf[16] = {0};
  for (int b = 0; b < 8; ++b) lenbuf[15 - b] = (unsigned char)(bits >> (8 * b));
  update(lenbuf, 16);
  for (int i = 0; i < 8; ++i) {
    const uint64_t v = __builtin_bswap64(st[i]);
    memcpy(out + 8 * i, &v, 8);
  }
}

void sha512_raw(const void* data, size_t len, unsigned char out[64]) {
  Sha512 s;
  s.update(data, len);
  s.final(out);
}

void to_hex(const unsigned char raw[64], char hex[128]) {
  static const char hx[] = "0123456789abcdef";
  for (int i = 0; i < 64; ++i) {
    hex[2 * i] = hx[raw[i] >> 4];
    hex[2 * i + 1] = hx[raw[i] & 15];
  }
}

void sha512_hex(const void* data, size_t len, char hex[128]) {
  unsigned char raw[64];
  sha512_raw(data, len, raw);
  to_hex(raw, hex);
}

}  // namespace nwk
