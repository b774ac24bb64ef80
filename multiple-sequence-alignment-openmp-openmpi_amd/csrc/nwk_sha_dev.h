// nwk_sha_dev.h -- device SHA-512 (FIPS 180-4) on register pairs, shared by
// nw_hash (nwk_hash.hip) and the bits kernels' fused per-pair finalize
// (nwk_bits.hip).  Reference: sw::sha512::calculate (sha512.hh:159-164).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nwk {
namespace shadev {

static __constant__ uint64_t kK512[80] = {
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

// 64-bit helpers on the 32-bit halves: a rotate by a constant is two
// v_alignbit_b32 (a generic 64-bit rotate compiled to two 64-bit shifts and two
// ORs), and every 3-input boolean function (XOR3, Ch, Maj) is one
// v_bitop3_b32 per half (truth tables over S0 = 0xF0, S1 = 0xCC, S2 = 0xAA).
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));  // {lo, hi}: a 64-bit value's halves in one register pair
template <int N>
__device__ __forceinline__ uint64_t rotr(uint64_t x) {
  const u32x2 v = __builtin_bit_cast(u32x2, x);
  u32x2 r;
  if constexpr (N < 32) {
    r.x = __builtin_amdgcn_alignbit(v.y, v.x, N);
    r.y = __builtin_amdgcn_alignbit(v.x, v.y, N);
  } else {
    r.x = __builtin_amdgcn_alignbit(v.x, v.y, N - 32);
    r.y = __builtin_amdgcn_alignbit(v.y, v.x, N - 32);
  }
  return __builtin_bit_cast(uint64_t, r);
}
template <unsigned F>
__device__ __forceinline__ uint64_t bop3(uint64_t a, uint64_t b, uint64_t c) {
  const u32x2 x = __builtin_bit_cast(u32x2, a), y = __builtin_bit_cast(u32x2, b), z = __builtin_bit_cast(u32x2, c);
  u32x2 r;
  r.x = __builtin_amdgcn_bitop3_b32(x.x, y.x, z.x, F);
  r.y = __builtin_amdgcn_bitop3_b32(x.y, y.y, z.y, F);
  return __builtin_bit_cast(uint64_t, r);
}
constexpr unsigned kXor3 = 0x96u, kCh = 0xCAu, kMaj = 0xE8u;

struct Sha {
  uint64_t s[8];
  __device__ void init() {
    s[0] = 0x6a09e667f3bcc908ULL; s[1] = 0xbb67ae8584caa73bULL; s[2] = 0x3c6ef372fe94f82bULL;
    s[3] = 0xa54ff53a5f1d36f1ULL; s[4] = 0x510e527fade682d1ULL; s[5] = 0x9b05688c2b3e6c1fULL;
    s[6] = 0x1f83d9abfb41bd6bULL; s[7] = 0x5be0cd19137e2179ULL;
  }
  // FIPS 180-4 6.4.2 on one 1024-bit block (big-endian words), rolling schedule
  __device__ void block(uint64_t (&w)[16]) {
    uint64_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll
    for (int t = 0; t < 80; ++t) {
      uint64_t wt;
      if (t < 16) {
        wt = w[t];
      } else {
        const uint64_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
        const uint64_t s0 = bop3<kXor3>(rotr<1>(w15), rotr<8>(w15), w15 >> 7);
        const uint64_t s1 = bop3<kXor3>(rotr<19>(w2), rotr<61>(w2), w2 >> 6);
        wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
        w[t & 15] = wt;
      }
      const uint64_t t1 = h + bop3<kXor3>(rotr<14>(e), rotr<18>(e), rotr<41>(e)) + bop3<kCh>(e, f, g) + kK512[t] + wt;
      const uint64_t t2 = bop3<kXor3>(rotr<28>(a), rotr<34>(a), rotr<39>(a)) + bop3<kMaj>(a, b, c);
      h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
  }
  // The same block with the rounds rolled by 16 (five trips): about half the
  // live registers of the fully unrolled form, for kernels that must stay at
  // <= 128 VGPRs (the bits kernels' fused finalize)
  __device__ void block_rolled(uint64_t (&w)[16]) {
    uint64_t a = s[0], b = s[1], c = s[2], d = s[3], e = s[4], f = s[5], g = s[6], h = s[7];
#pragma unroll 1
    for (int t0 = 0; t0 < 80; t0 += 16) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        if (t0 > 0) {
          const uint64_t w15 = w[(q + 1) & 15], w2 = w[(q + 14) & 15];
          const uint64_t s0 = bop3<kXor3>(rotr<1>(w15), rotr<8>(w15), w15 >> 7);
          const uint64_t s1 = bop3<kXor3>(rotr<19>(w2), rotr<61>(w2), w2 >> 6);
          w[q] = w[q] + s0 + w[(q + 9) & 15] + s1;
        }
        const uint64_t t1 = h + bop3<kXor3>(rotr<14>(e), rotr<18>(e), rotr<41>(e)) + bop3<kCh>(e, f, g) + kK512[t0 + q] + w[q];
        const uint64_t t2 = bop3<kXor3>(rotr<28>(a), rotr<34>(a), rotr<39>(a)) + bop3<kMaj>(a, b, c);
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
      }
    }
    s[0] += a; s[1] += b; s[2] += c; s[3] += d; s[4] += e; s[5] += f; s[6] += g; s[7] += h;
  }
};

__device__ __forceinline__ uint64_t hex16(uint32_t v) {  // 8 nibbles of v -> 8 ASCII bytes, big-endian word
  uint64_t o = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const unsigned nib = (v >> (28 - 4 * k)) & 15u;
    o = (o << 8) | (nib < 10 ? '0' + nib : 'a' + nib - 10);
  }
  return o;
}

// inclusive wave scan (64 lanes)
__device__ __forceinline__ unsigned wave_incl_scan(unsigned v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned u = (unsigned)__shfl_up((int)v, o);
    v += lane >= o ? u : 0u;
  }
  return v;
}

}  // namespace shadev
}  // namespace nwk
