// Chain-link microbenchmark (skel:159 chain): the reference-style sha512_hex of the
// 256-byte concatenation vs the engine chain_step with precomputed schedules.
// build: g++ -O3 -I../../multiple-sequence-alignment-openmp-openmpi_amd/csrc chain_probe.cpp ../../multiple-sequence-alignment-openmp-openmpi_amd/csrc/sha512.cpp -o chain_probe
#include <chrono>
#include <cstdio>
#include <cstring>
#include <cstdint>
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
// hex chars of the 8 nibbles of x (32 bits), most significant first, as a big-endian word
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
#define RND(a, b, c, d, e, f, g, h, kw)                                   \
  do {                                                                \
    const uint64_t t1 = h + S1(e) + (g ^ (e & (f ^ g))) + (kw);        \
    const uint64_t t2 = S0(a) + ((a & b) | (c & (a | b)));             \
    d += t1;                                                          \
    h = t1 + t2;                                                      \
  } while (0)
// compress with a full precomputed K+W schedule
static inline void comp_kw(uint64_t st[8], const uint64_t* kw) {
  uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  for (int t = 0; t < 80; t += 8) {
    RND(a, b, c, d, e, f, g, h, kw[t + 0]); RND(h, a, b, c, d, e, f, g, kw[t + 1]);
    RND(g, h, a, b, c, d, e, f, kw[t + 2]); RND(f, g, h, a, b, c, d, e, kw[t + 3]);
    RND(e, f, g, h, a, b, c, d, kw[t + 4]); RND(d, e, f, g, h, a, b, c, kw[t + 5]);
    RND(c, d, e, f, g, h, a, b, kw[t + 6]); RND(b, c, d, e, f, g, h, a, kw[t + 7]);
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
  // reference chain
  auto t0 = std::chrono::steady_clock::now();
  char buf[256]; size_t la = 0;
  for (int p = 0; p < P; ++p) { to_hex(ph.data() + 64 * p, buf + la); char acc[128]; sha512_hex(buf, la + 128, acc); memcpy(buf, acc, 128); la = 128; }
  auto t1 = std::chrono::steady_clock::now();
  // fast chain: block 2 schedule per link (precomputed), block 3 const
  std::vector<uint64_t> kw2((size_t)P * 80);
  auto t2a = std::chrono::steady_clock::now();
  for (int p = 0; p < P; ++p) {
    uint64_t w16[16];
    for (int q = 0; q < 8; ++q) {
      uint64_t v; memcpy(&v, ph.data() + 64 * p + 8 * q, 8); v = __builtin_bswap64(v);
      w16[2 * q] = hexword(v >> 32); w16[2 * q + 1] = hexword(v);
    }
    sched(w16, kw2.data() + 80 * (size_t)p);
  }
  auto t2b = std::chrono::steady_clock::now();
  uint64_t kw3[80], w16p[16] = {0x8000000000000000ULL};
  w16p[15] = 256 * 8;
  sched(w16p, kw3);
  uint64_t dig[8]; bool first = true;
  auto t2 = std::chrono::steady_clock::now();
  for (int p = 0; p < P; ++p) {
    uint64_t st[8]; memcpy(st, IV, 64);
    if (first) {  // acc == "": message = hex(ph) only (128 B) -> blocks: hex, pad(len 1024)
      uint64_t w16[16] = {0x8000000000000000ULL}; w16[15] = 128 * 8; uint64_t kwp[80]; sched(w16, kwp);
      comp_kw(st, kw2.data()); comp_kw(st, kwp); first = false;
    } else {
      uint64_t w16[16];
      for (int q = 0; q < 8; ++q) { w16[2 * q] = hexword(dig[q] >> 32); w16[2 * q + 1] = hexword(dig[q]); }
      uint64_t kw1[80]; sched(w16, kw1);
      comp_kw(st, kw1); comp_kw(st, kw2.data() + 80 * (size_t)p); comp_kw(st, kw3);
    }
    memcpy(dig, st, 64);
  }
  auto t3 = std::chrono::steady_clock::now();
  char hx[129]; for (int q = 0; q < 8; ++q) { uint64_t a = hexword(dig[q] >> 32), b = hexword(dig[q]); for (int i = 0; i < 8; ++i) { hx[16*q+i] = (char)(a >> (56 - 8*i)); hx[16*q+8+i] = (char)(b >> (56-8*i)); } }
  hx[128] = 0;
  printf("ref  %.3f ms (%.1f ns/link)\n", std::chrono::duration<double, std::milli>(t1 - t0).count(), std::chrono::duration<double, std::nano>(t1 - t0).count() / P);
  printf("pre  %.3f ms (block-2 schedules, parallelizable)\n", std::chrono::duration<double, std::milli>(t2b - t2a).count());
  printf("fast %.3f ms (%.1f ns/link)\n", std::chrono::duration<double, std::milli>(t3 - t2).count(), std::chrono::duration<double, std::nano>(t3 - t2).count() / P);
  printf("match %d\n", memcmp(hx, buf, 128) == 0);
}
