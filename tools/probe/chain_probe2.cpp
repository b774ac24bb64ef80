// Chain-link A/B (skel:159): the engine's chain_step (csrc/sha512.cpp) against a
// variant that rolls block 1's message schedule into its rounds and carries
// Maj's (a ^ b) to the next round.  Both over the same 32,640 problemhashes;
// prints ns per link and whether the answers agree.
// build: g++ -O3 -march=x86-64-v3 -I../../multiple-sequence-alignment-openmp-openmpi_amd/csrc chain_probe2.cpp ../../multiple-sequence-alignment-openmp-openmpi_amd/csrc/sha512.cpp -o chain_probe2
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "sha512.h"
using namespace nwk;

static const uint64_t K[80] = {
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
static const uint64_t IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                               0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                               0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
static inline uint64_t ror(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
static inline uint64_t hexword(uint64_t x) {
  x &= 0xffffffffULL;
  x = (x | (x << 16)) & 0x0000FFFF0000FFFFULL;
  x = (x | (x << 8)) & 0x00FF00FF00FF00FFULL;
  x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0FULL;
  const uint64_t gt9 = ((x + 0x0606060606060606ULL) >> 4) & 0x0101010101010101ULL;
  return x + 0x3030303030303030ULL + gt9 * 0x27;
}
#define S0(x) (ror(x, 28) ^ ror(x, 34) ^ ror(x, 39))
#define S1(x) (ror(x, 14) ^ ror(x, 18) ^ ror(x, 41))
#define s0(x) (ror(x, 1) ^ ror(x, 8) ^ ((x) >> 7))
#define s1(x) (ror(x, 19) ^ ror(x, 61) ^ ((x) >> 6))
// Maj through the carried (a ^ b): Maj(a, b, c) = b ^ ((a ^ b) & (b ^ c))
#define RND(a, b, c, d, e, f, g, h, kw, AB, BC)                   \
  do {                                                            \
    const uint64_t t1 = (h + (kw)) + (g ^ (e & (f ^ g))) + S1(e); \
    AB = a ^ b;                                                   \
    d += t1;                                                      \
    h = t1 + (S0(a) + (b ^ (AB & BC)));                           \
  } while (0)
static inline void comp_kw(uint64_t st[8], const uint64_t* kw) {
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  uint64_t x = b ^ c, y;
  for (int t = 0; t < 80; t += 8) {
    RND(a, b, c, d, e, f, g, h, kw[t + 0], y, x); RND(h, a, b, c, d, e, f, g, kw[t + 1], x, y);
    RND(g, h, a, b, c, d, e, f, kw[t + 2], y, x); RND(f, g, h, a, b, c, d, e, kw[t + 3], x, y);
    RND(e, f, g, h, a, b, c, d, kw[t + 4], y, x); RND(d, e, f, g, h, a, b, c, kw[t + 5], x, y);
    RND(c, d, e, f, g, h, a, b, kw[t + 6], y, x); RND(b, c, d, e, f, g, h, a, kw[t + 7], x, y);
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}
// block 1 from its 16 words, schedule rolled into the rounds
static inline void comp_w(uint64_t st[8], uint64_t w[16]) {
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  uint64_t x = b ^ c, y;
  for (int t = 0; t < 80; t += 8) {
    if (t >= 16)
      for (int q = 0; q < 8; ++q) {
        const int u = t + q;
        w[u & 15] += s1(w[(u - 2) & 15]) + w[(u - 7) & 15] + s0(w[(u - 15) & 15]);
      }
    RND(a, b, c, d, e, f, g, h, K[t + 0] + w[(t + 0) & 15], y, x); RND(h, a, b, c, d, e, f, g, K[t + 1] + w[(t + 1) & 15], x, y);
    RND(g, h, a, b, c, d, e, f, K[t + 2] + w[(t + 2) & 15], y, x); RND(f, g, h, a, b, c, d, e, K[t + 3] + w[(t + 3) & 15], x, y);
    RND(e, f, g, h, a, b, c, d, K[t + 4] + w[(t + 4) & 15], y, x); RND(d, e, f, g, h, a, b, c, K[t + 5] + w[(t + 5) & 15], x, y);
    RND(c, d, e, f, g, h, a, b, K[t + 6] + w[(t + 6) & 15], y, x); RND(b, c, d, e, f, g, h, a, K[t + 7] + w[(t + 7) & 15], x, y);
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}
static inline void sched(const uint64_t w16[16], uint64_t kw[80]) {
  uint64_t w[80];
  for (int t = 0; t < 16; ++t) w[t] = w16[t];
  for (int t = 16; t < 80; ++t) w[t] = s1(w[t - 2]) + w[t - 7] + s0(w[t - 15]) + w[t - 16];
  for (int t = 0; t < 80; ++t) kw[t] = K[t] + w[t];
}
int main() {
  const int P = 32640;
  std::vector<unsigned char> ph(64 * (size_t)P);
  for (size_t i = 0; i < ph.size(); ++i) ph[i] = (unsigned char)(i * 2654435761u >> 13);
  std::vector<uint64_t> kw2((size_t)P * 80);
  for (int p = 0; p < P; ++p) chain_schedule(ph.data() + 64 * p, kw2.data() + 80 * (size_t)p);
  uint64_t kw3[80], w16p[16] = {0x8000000000000000ULL};
  w16p[15] = 256 * 8;
  sched(w16p, kw3);
  for (int rep = 0; rep < 3; ++rep) {
    ChainAcc acc;
    auto t0 = std::chrono::steady_clock::now();
    for (int p = 0; p < P; ++p) chain_step(&acc, kw2.data() + 80 * (size_t)p);
    auto t1 = std::chrono::steady_clock::now();
    // variant (the first link has no accumulator: same as chain_step's empty case)
    uint64_t dig[8];
    {
      ChainAcc a1;
      chain_step(&a1, kw2.data());
      memcpy(dig, a1.dig, 64);
    }
    auto t2 = std::chrono::steady_clock::now();
    for (int p = 1; p < P; ++p) {
      uint64_t st[8], w[16];
      memcpy(st, IV, 64);
      for (int q = 0; q < 8; ++q) { w[2 * q] = hexword(dig[q] >> 32); w[2 * q + 1] = hexword(dig[q]); }
      comp_w(st, w);
      comp_kw(st, kw2.data() + 80 * (size_t)p);
      comp_kw(st, kw3);
      memcpy(dig, st, 64);
    }
    auto t3 = std::chrono::steady_clock::now();
    printf("chain_step %.1f ns/link | variant %.1f ns/link | same %d\n",
           std::chrono::duration<double, std::nano>(t1 - t0).count() / P,
           std::chrono::duration<double, std::nano>(t3 - t2).count() / P, memcmp(dig, acc.dig, 64) == 0);
  }
}
