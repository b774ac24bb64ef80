// nwk_col.hip -- column-wise bit-parallel fill (mode kCol, kernel nw_align_col)
// for the reference's linear-gap recurrence (skel:211-226, sub:478-487) with
// pxy >= 0, pgap in {1, 2} and at most four distinct symbols: the domain of
// nw_align_bits, with a pair's critical path cut from m + n anti-diagonal
// steps to about n + m / 32.
//
// Recurrence down a column.  In G-space gaps cost 0, so down
// column j the horizontal differences h(i) = G[i][j-1] - G[i][j] obey
//     h(i) = max(e(i), h(i-1) - L(i)),   e(i) = max(S(i) - L(i), 0),
// L(i) = v(i, j-1) the previous column's vertical difference and S = 2 pgap
// (match) or 2 pgap - pxy (mismatch).  With thermometer planes t_k = [h > k]
// (k < NP = 2 pgap) and l_d = [L > d] this is, level by level from the top,
//     t_k(i) = G_k(i) | (P(i) & t_k(i-1)),   P = ~l_0,
//     G_k = (match & ~l_{NP-1-k}) | ~l_{SR-1-k} | OR_{d>=1} (~l_d & t_{k+d}(i-1))
// (SR = 2 pgap - pxy, ~l_{<0} = 0): a carry chain per level, resolved for 32
// rows at once by one add -- A = P | G_k, B = G_k, S = A + B + cin gives the
// carries c_i = G_i | (P_i & c_{i-1}) = t_k(i), and S ^ A ^ B = the carries
// shifted up one row, exactly the planes U_k = t_k(i-1) = h(i-1, j) the rest
// of the cell needs.  D = max(S, U, L) and v = D - U are nw_align_bits' plane
// algebra; the stored traceback bits are the same (diag = match | D == S_mm,
// up = [v == 0], skel:229-262's DIAG > UP > LEFT).
//
// Layout.  Bit b of lane t is row 32 t + b of a 2048-row band, and at step s
// lane t works on column s - t: a column's 32-row words pass down the wave one
// lane per step.  A lane's carry into its row 32 t comes from lane t - 1's
// carry out of the previous step (same column): v_addc_co_u32 takes the carry
// in and gives the carry out as 64-lane masks in SGPRs, so the hop to the next
// lane is one scalar shift.  Lane 0 takes the band above's last row instead
// (one bit per step from 32-column granules {epoch:32 | 32 plane bits}), and
// lane 63's carries out are the band's last row for the band below, collected
// by a scalar shift register and published per 32 columns.  A band therefore
// trails the band above by ~96 steps instead of nw_align_bits' 2112, and a
// pair's span is n + ~96 x bands steps.
//
// Stored layout per band: nw_align_bits' 8-step blocks (1024 dwords; diag
// bits of step s, lane t at B * 1024 + ((s & 7) >> 2) * 256 + 4 t + (s & 3),
// up bits 512 dwords further), here holding column s - t, rows 32 t .. + 31.
// Windowed storage keeps bits_nblk blocks from bits_blk_lo(band) on: every
// step with a cell within bits_w columns of the diagonal j = i n / m.
#include "nwk_bits_dev.h"

namespace nwk {
namespace {

// v_addc_co_u32 with the carry as a 64-lane SGPR mask: c in = lane t's carry
// in, c out = lane t's carry out
__device__ __forceinline__ unsigned col_addc(unsigned a, unsigned b, u64& c) {
  unsigned s;
  asm("v_addc_co_u32 %0, %1, %2, %3, %1" : "=v"(s), "+s"(c) : "v"(a), "v"(b));
  // (an empty scalar asm on the carry: the optimizer would otherwise carry the
  // asm's {vgpr, sgpr} result pair through loop phis, making the carry per-lane)
  asm("" : "+s"(c));
  return s;
}

// The carries' hop to the next lane, on the scalar unit (written out so the
// compiler keeps it there): c = (c << 1) | the band above's bit QQ of this half
// (lane 0's carry in), and lane 63's carry out of the previous step (bit 63 of
// the old c) enters the band's last-row shift register acc.  One SCC chain, 4
// SALU: SCC = inj bit QQ; lo = 2 lo + SCC (SCC = old bit 31); hi = 2 hi + SCC
// (SCC = old bit 63); acc = 2 acc + SCC.  (Was 5: a 64-bit shift, a bit
// extract and an OR for c, a bit test and an add for acc.)
template <int QQ>
__device__ __forceinline__ void col_hop(u64& c, unsigned& acc, u64 inj) {
  unsigned lo = (unsigned)c, hi = (unsigned)(c >> 32);
  asm("s_bitcmp1_b64 %[inj], %[pos]\n\t"
      "s_addc_u32 %[lo], %[lo], %[lo]\n\t"
      "s_addc_u32 %[hi], %[hi], %[hi]\n\t"
      "s_addc_u32 %[acc], %[acc], %[acc]"
      : [lo] "+s"(lo), [hi] "+s"(hi), [acc] "+s"(acc)
      : [inj] "s"(inj), [pos] "i"(QQ)
      : "scc");
  c = ((u64)hi << 32) | lo;
}

// G_K's middle terms OR_{d = D .. I-1} (~l_d & T_{K+d})
template <int NP, int K, int D, int I>
__device__ __forceinline__ unsigned col_mid(unsigned G, const unsigned (&l)[NP], const unsigned (&T)[NP]) {
  if constexpr (D >= I) {
    return G;
  } else {
    G = BOP3(G, l[D], T[K + D], kA | (~kB & kC));
    return col_mid<NP, K, D + 1, I>(G, l, T);
  }
}

// Level K: resolves t_K for this lane's 32 rows; T[K] = t_K shifted up one row
// (bit 0 = the carry in), cout = this lane's carry out (t_K of its row 31)
template <int NP, int SR, int K>
__device__ __forceinline__ void col_level(unsigned match, unsigned P, const unsigned (&l)[NP], unsigned (&T)[NP],
                                          u64& c) {
  constexpr int J = SR - 1 - K;  // mismatch term ~l_J (none below 0)
  constexpr int I = NP - 1 - K;  // match term ~l_I
  unsigned G;
  if constexpr (J >= I) {
    G = ~l[J];  // ~l_I and every ~l_d with d <= I lie inside ~l_J
  } else {
    if constexpr (K == NP - 1) G = BOP3(match, l[0], l[0], kA & ~kB);  // match & ~l_0
    else G = BOP3(l[I], match, T[NP - 1], ~kA & (kB | kC));           // ~l_I & (match | T_{NP-1})
    constexpr int D0 = J + 1 > 1 ? J + 1 : 1;  // terms d <= J lie inside ~l_J
    G = col_mid<NP, K, D0, I>(G, l, T);
    if constexpr (J >= 0) G = BOP3(G, l[J], l[J], kA | ~kB);  // | ~l_J
  }
  if constexpr (J >= 0) {  // P = ~l_0 lies inside G: t_K = G, no carry chain
    T[K] = col_addc(G, G, c);
  } else {
    const unsigned A = K == NP - 1 ? P : (P | G);  // (level NP-1: G inside P)
    const unsigned S = col_addc(A, G, c);
    T[K] = BOP3(S, A, G, kA ^ kB ^ kC);
  }
}

template <int NP, int SR, int K>
__device__ __forceinline__ void col_levels(unsigned match, unsigned P, const unsigned (&l)[NP], unsigned (&T)[NP],
                                           u64 (&c)[NP]) {
  col_level<NP, SR, K>(match, P, l, T, c[K]);
  if constexpr (K > 0) col_levels<NP, SR, K - 1>(match, P, l, T, c);
}

template <int NP, int QQ, int K = 0>
__device__ __forceinline__ void col_hops(u64 (&c)[NP], unsigned (&acc)[NP], const u64 (&inj)[NP]) {
  col_hop<QQ>(c[K], acc[K], inj[K]);
  if constexpr (K + 1 < NP) col_hops<NP, QQ, K + 1>(c, acc, inj);
}

// Eight steps s0 .. s0+7 (s0 % 8 == 0) of one band.
//   x0, x1   code bit planes of this lane's 32 rows
//   w0, w1   y window of this 32-step half (bit 31 - q = code of column s_half + q - lane)
//   l        v planes of this lane's previous column
//   c        per level: the carries out of the previous step (64-lane masks)
//   acc      shift registers of lane 63's carries out (the band's last row)
//   inj      the band above's last row for lane 0's columns of this half (bit q = column s_half + q)
//   pub      CAP: acc after step s_half + 30's carries (columns s_half - 94 .. s_half - 63)
//   MASK     steps of the first super-block: columns < 0 keep v = 0 (the left border)
//   END      steps that may hold column capc = n - 1: lane t = s - capc holds it;
//            the scalar unit reads its vertical differences (v_readlane) and adds
//            those of its rows < m (nvr0 - 32 t of them) to cnt (the fill-vs-walk
//            guard's end value, FillArgs::endv).  All scalar: no VGPR lives
//            across the loop for it (a per-lane mask and counter did, and the
//            96-VGPR instantiation spilled ~270 registers: C3 145 -> 172 ms)
template <int NP, int SR, bool MASK, bool CAP, int BLK, bool END>
__device__ __forceinline__ void col_block(int s0, int lane, unsigned x0, unsigned x1, unsigned w0, unsigned w1,
                                          unsigned (&l)[NP], u64 (&c)[NP], unsigned (&acc)[NP],
                                          const u64 (&inj)[NP], unsigned (&pub)[NP], unsigned* st, bool sto,
                                          int capc, int nvr0, int& cnt) {
  unsigned dw[8], uw[8];
  auto step = [&](auto qc) {
    constexpr int q = decltype(qc)::value;
    constexpr int qq = 8 * BLK + q;  // step s0 + q within its 32-step half
    const int s = s0 + q;
    const unsigned Y0 = (unsigned)((int)(w0 << qq) >> 31);  // code bits of column s - lane, as 0 / ~0
    const unsigned Y1 = (unsigned)((int)(w1 << qq) >> 31);
    const unsigned match = BOP3(x0 ^ Y0, x1, Y1, ~(kA | (kB ^ kC)));  // ~((x0^Y0) | (x1^Y1))
    col_hops<NP, qq>(c, acc, inj);
    if constexpr (CAP && q == 7) {
#pragma unroll
      for (int k = 0; k < NP; ++k) pub[k] = acc[k];
    }
    unsigned T[NP], D[NP], Vn[NP];
    const unsigned P = ~l[0];
    col_levels<NP, SR, NP - 1>(match, P, l, T, c);
#pragma unroll
    for (int k = 0; k < NP; ++k) D[k] = k < SR ? ~0u : BOP3(match, T[k], l[k], kA | kB | kC);
    bits_diffs<NP, SR>(T, D, Vn);  // v = D - U, U = T
    if constexpr (MASK) {
      const bool live = s >= lane;  // column s - lane >= 0
#pragma unroll
      for (int k = 0; k < NP; ++k) Vn[k] = live ? Vn[k] : 0u;
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) l[k] = Vn[k];
    if constexpr (END) {
      const int t = s - capc;  // (uniform) the lane at column capc
      if ((unsigned)t < 64u) {
        const int nv = nvr0 - 32 * t;
        const unsigned mk = nv >= 32 ? ~0u : (nv <= 0 ? 0u : (1u << nv) - 1u);
#pragma unroll
        for (int k = 0; k < NP; ++k) cnt += __builtin_popcount((unsigned)__builtin_amdgcn_readlane((int)Vn[k], t) & mk);
      }
    }
    if constexpr (SR < 0) dw[q] = match;
    else if constexpr (SR >= NP) dw[q] = ~0u;
    else dw[q] = BOP3(match, D[SR], D[SR], kA | ~kB);  // match | ~D_SR
    uw[q] = Vn[0];  // stored raw: UP is v == 0 (bit clear)
    if constexpr ((q & 3) == 3) {
      typedef unsigned u4 __attribute__((ext_vector_type(4)));
      constexpr int h = q >> 2;
      if (sto) {
        __builtin_nontemporal_store(u4{dw[4 * h], dw[4 * h + 1], dw[4 * h + 2], dw[4 * h + 3]},
                                    reinterpret_cast<u4*>(st + 256 * h));
        __builtin_nontemporal_store(u4{uw[4 * h], uw[4 * h + 1], uw[4 * h + 2], uw[4 * h + 3]},
                                    reinterpret_cast<u4*>(st + 512 + 256 * h));
      }
    }
  };
  step(std::integral_constant<int, 0>{});
  step(std::integral_constant<int, 1>{});
  step(std::integral_constant<int, 2>{});
  step(std::integral_constant<int, 3>{});
  step(std::integral_constant<int, 4>{});
  step(std::integral_constant<int, 5>{});
  step(std::integral_constant<int, 6>{});
  step(std::integral_constant<int, 7>{});
}

// every active lane's p (a uniform result the compiler can see as one)
__device__ __forceinline__ bool wall(bool p) { return __builtin_amdgcn_ballot_w64(!p) == 0ull; }

// lane `sel`'s word of v := x (uniform x, sel)
__device__ __forceinline__ unsigned writelane(unsigned v, int x, int sel) {
  // (two scalar operands: the lane select goes through m0, the constant bus takes one SGPR)
  asm volatile("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0" : "+v"(v)
               : "s"(__builtin_amdgcn_readfirstlane(x)), "s"(__builtin_amdgcn_readfirstlane(sel)) : "m0");
  return v;
}

// s_ff1 of a uniform 64-bit mask (forced into SGPRs: a loop variable the
// compiler keeps in VGPRs on some path would otherwise make the asm operand illegal)
__device__ __forceinline__ int sff1u(u64 m) {
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)m), hi = __builtin_amdgcn_readfirstlane((unsigned)(m >> 32));
  return sff1(((u64)hi << 32) | lo);
}

// windowed storage: a lane's words of an 8-step block (dev = c m - i n over
// them spans [hi - 7 m - 31 n, hi]) are stored iff that span meets
// [-lim, lim], lim = bits_w m; hlim = lim + 7 m + 31 n
__device__ __forceinline__ bool bits_lane_stored(int64_t hi, int64_t lim, int64_t hlim) {
  return hi >= -lim && hi <= hlim;
}

__device__ __forceinline__ int smax(int a, int b) {
  int r;
  asm("s_max_i32 %0, %1, %2" : "=s"(r) : "s"(__builtin_amdgcn_readfirstlane(a)), "s"(__builtin_amdgcn_readfirstlane(b)) : "scc");
  return r;
}

// The run loop of a pass without window checks, as one block of scalar code
// (the compiled loop spends ~65 instructions and 8 branches on a stop, this
// one ~25): the walk of trace_col's `walk` lambda, step for step.
//   loop:  bnd = min(K - trowlo, LL); L > bnd or K - Kb > 31: done
//          Dm, Um = the key's D and U lanes (v_bfe + v_cmp per mask)
//          ls = min(ff1(~Dm & -1 << L), bnd + 1); ls > bnd: L = ls, done (a D run)
//          U at ls: down lane ls's column (readlane of WD, WU): U^nU, then D
//          (K = Kb + j, loop) or L (finL[ls], K = Kb + j + 1, lrun), or the run
//          leaves the window (L = ls, K = Kb + jlo - 1, done)
//          else L at ls: finL[ls], L = ls + 1, K + 1, lrun
//   lrun:  rr = K - L; lend = min(LL, 31 + Kb - rr) + 1; L >= lend: loop
//          le = min(ff1(~Lm & -1 << L), lend) over the row's L cells (WL at bit rr - Kb + lane)
//          finL |= bits L .. le - 1; L = le; K = rr + le; loop
__device__ __forceinline__ void walk_asm(unsigned WD, unsigned WU, unsigned WL, int lane, int Kb, int trowlo, int LL,
                                         int& K, int& L, u64& finL, unsigned& nUv, int& maxU) {
  int bnd, i, ls, t, j, nU;
  unsigned wd, wu, sm;
  u64 Dm, Um, m64;
  unsigned vt;
  asm volatile(
      "s_nop 1\n"
      "Lwloop%=:\n\t"
      "s_sub_i32 %[bnd], %[K], %[trowlo]\n\t"
      "s_min_i32 %[bnd], %[bnd], %[LL]\n\t"
      "s_cmp_gt_i32 %[L], %[bnd]\n\t"
      "s_cbranch_scc1 Lwdone%=\n\t"
      "s_sub_i32 %[i], %[K], %[Kb]\n\t"
      "s_cmp_gt_u32 %[i], 31\n\t"
      "s_cbranch_scc1 Lwdone%=\n\t"
      "v_bfe_u32 %[vt], %[WD], %[i], 1\n\t"
      "v_cmp_ne_u32_e64 %[Dm], 0, %[vt]\n\t"
      "v_bfe_u32 %[vt], %[WU], %[i], 1\n\t"
      "v_cmp_eq_u32_e64 %[Um], 0, %[vt]\n\t"
      "s_lshl_b64 %[m64], -1, %[L]\n\t"
      "s_andn2_b64 %[m64], %[m64], %[Dm]\n\t"
      "s_ff1_i32_b64 %[ls], %[m64]\n\t"
      "s_add_i32 %[t], %[bnd], 1\n\t"
      "s_min_u32 %[ls], %[ls], %[t]\n\t"
      "s_cmp_gt_i32 %[ls], %[bnd]\n\t"
      "s_cbranch_scc1 Lwdrun%=\n\t"
      "s_bitcmp1_b64 %[Um], %[ls]\n\t"
      "s_cbranch_scc1 Lwup%=\n\t"
      // an L move at ls
      "s_bitset1_b64 %[finL], %[ls]\n\t"
      "s_add_i32 %[L], %[ls], 1\n\t"
      "s_add_i32 %[K], %[K], 1\n\t"
      "s_branch Lwlrun%=\n"
      "Lwup%=:\n\t"
      // a U move, then down lane ls's column while D is clear and U set
      "v_readlane_b32 %[wd], %[WD], %[ls]\n\t"
      "v_readlane_b32 %[wu], %[WU], %[ls]\n\t"
      "s_add_i32 %[j], %[trowlo], %[ls]\n\t"
      "s_sub_i32 %[j], %[j], %[Kb]\n\t"
      "s_max_i32 %[j], %[j], 0\n\t"               // jlo
      "s_lshl_b32 %[t], 2, %[i]\n\t"
      "s_add_i32 %[t], %[t], -1\n\t"               // bits 0 .. i (2 << 31 wraps to 0: all)
      "s_or_b32 %[sm], %[wd], %[wu]\n\t"
      "s_and_b32 %[sm], %[sm], %[t]\n\t"
      "s_lshl_b32 %[t], -1, %[j]\n\t"
      "s_and_b32 %[sm], %[sm], %[t]\n\t"
      "s_cmp_eq_u32 %[sm], 0\n\t"
      "s_cbranch_scc1 Lwuleave%=\n\t"
      "s_flbit_i32_b32 %[t], %[sm]\n\t"
      "s_sub_i32 %[j], 31, %[t]\n\t"               // j: the key the vertical run stops at
      "s_sub_i32 %[nU], %[i], %[j]\n\t"
      "s_mov_b32 m0, %[ls]\n\t"
      "v_writelane_b32 %[nUv], %[nU], m0\n\t"
      "s_max_i32 %[maxU], %[maxU], %[nU]\n\t"
      "s_add_i32 %[L], %[ls], 1\n\t"
      "s_add_i32 %[K], %[Kb], %[j]\n\t"
      "s_bitcmp1_b32 %[wd], %[j]\n\t"
      "s_cbranch_scc1 Lwloop%=\n\t"                // ... then D
      "s_bitset1_b64 %[finL], %[ls]\n\t"          // ... then L
      "s_add_i32 %[K], %[K], 1\n"
      "Lwlrun%=:\n\t"
      // a horizontal run on row rr = K - L: the row's cells that move L, one ballot
      "s_sub_i32 %[t], %[K], %[L]\n\t"             // rr
      "s_sub_i32 %[j], %[Kb], %[t]\n\t"
      "s_add_i32 %[j], %[j], 31\n\t"
      "s_min_i32 %[j], %[j], %[LL]\n\t"
      "s_add_i32 %[j], %[j], 1\n\t"                // lend
      "s_cmp_ge_i32 %[L], %[j]\n\t"
      "s_cbranch_scc1 Lwloop%=\n\t"
      "s_sub_i32 %[nU], %[t], %[Kb]\n\t"
      "v_add_u32_e32 %[vt], %[nU], %[lane]\n\t"
      "v_bfe_u32 %[vt], %[WL], %[vt], 1\n\t"
      "v_cmp_ne_u32_e64 %[Dm], 0, %[vt]\n\t"
      "s_lshl_b64 %[m64], -1, %[L]\n\t"
      "s_andn2_b64 %[m64], %[m64], %[Dm]\n\t"
      "s_ff1_i32_b64 %[ls], %[m64]\n\t"
      "s_min_u32 %[ls], %[ls], %[j]\n\t"           // le
      "s_sub_i32 %[nU], %[ls], %[L]\n\t"
      "s_bfm_b64 %[m64], %[nU], %[L]\n\t"          // lanes L .. le - 1
      "s_or_b64 %[finL], %[finL], %[m64]\n\t"
      "s_mov_b32 %[L], %[ls]\n\t"
      "s_add_i32 %[K], %[t], %[ls]\n\t"
      "s_branch Lwloop%=\n"
      "Lwuleave%=:\n\t"
      // the vertical run leaves the tile's rows (or the key window): U moves down to there
      "s_sub_i32 %[nU], %[i], %[j]\n\t"
      "s_add_i32 %[nU], %[nU], 1\n\t"
      "s_mov_b32 m0, %[ls]\n\t"
      "v_writelane_b32 %[nUv], %[nU], m0\n\t"
      "s_max_i32 %[maxU], %[maxU], %[nU]\n\t"
      "s_mov_b32 %[L], %[ls]\n\t"
      "s_add_i32 %[K], %[Kb], %[j]\n\t"
      "s_add_i32 %[K], %[K], -1\n\t"
      "s_branch Lwdone%=\n"
      "Lwdrun%=:\n\t"
      "s_mov_b32 %[L], %[ls]\n"
      "Lwdone%=:"
      : [K] "+s"(K), [L] "+s"(L), [finL] "+s"(finL), [nUv] "+v"(nUv), [maxU] "+s"(maxU), [bnd] "=&s"(bnd),
        [i] "=&s"(i), [ls] "=&s"(ls), [t] "=&s"(t), [j] "=&s"(j), [nU] "=&s"(nU), [wd] "=&s"(wd), [wu] "=&s"(wu),
        [sm] "=&s"(sm), [Dm] "=&s"(Dm), [Um] "=&s"(Um), [m64] "=&s"(m64), [vt] "=&v"(vt)
      : [WD] "v"(WD), [WU] "v"(WU), [WL] "v"(WL), [lane] "v"(lane), [Kb] "s"(Kb), [trowlo] "s"(trowlo), [LL] "s"(LL)
      : "scc", "m0");
}

// Traceback of one pair from (m, n) over the stored (diag, up) bits
// (SPEC = false), or a speculative segment of band sb (SPEC = true, below).
//
// Tiles are 64 columns (lane L holds column cts - L) by four row-lanes ta ..
// ta - 3 (128 rows), eight dwords per lane: each lane loads its column's words
// at steps column + row-lane.  A D move goes from (row r, lane L) to (r - 1,
// L + 1), so every cell of a diagonal run has the same key K = r + L; a U move
// stays in the lane (key K - 1), an L move goes to lane L + 1 (key K + 1).
// Each lane re-indexes its column of bits by key once per tile (a funnel
// shift), then the walk runs on the scalar unit: one ballot pair per new key
// gives every lane's D and U bit on that key's diagonal; a D run stops at the
// first lane >= L whose D bit is clear (s_ff1); a stop that moves U continues
// down its lane's column (a vertical run read from that lane's key window by
// v_readlane) until a cell moves D or L.  Per lane the moves are U^nU then one
// D or L, written once per tile (prefix sum of the lanes' move counts) through
// a 1 KB LDS ring flushed to ops[].  Storage bound: a cell is read only when
// its column is >= the band's lowest stored step (then its step, column +
// row-lane, is stored too); a walk that leaves flags the pair for a re-run
// with full storage.
//
// Segmented traceback (pd.spec_every > 0).  A walk is one wave's chain of
// dependent scalar steps, ~0.1 us per move on a busy chip: a 35k x 90k pair of
// big13 took 7-11 ms, all of it after the pair's last band filled.  So every
// band b but the last, once filled, traces a speculative segment of its own
// rows (SPEC): from its last row at a guessed column up to the band's top,
// recording for each row the cell it entered the row at and its move index
// (recs, epoch-tagged).  Traceback paths from different cells merge and then
// coincide (the walk is deterministic), so the pair's own walk (from (m, n),
// on the wave that filled the last band) checks at each pass start whether its
// cell lies on band b's segment -- row r's entry column c_hi and the row's L
// moves give the segment's cells on r -- and on a hit copies the segment's
// remaining moves and jumps to its exit: the walk then only crosses the rows
// from a band's bottom to the merge.  A segment that fails (left the stored
// window) is never merged into; a band whose segment never merges is walked
// in full, as before.
// WIN: the pair has windowed storage (pd.bits_w > 0); without it the checked
// walk is compiled out (its merge with the asm walk made the compiler
// materialize an undefined phi input as a v_readfirstlane of the next tile's
// load register, and so wait for that load on every pass)
template <bool SPEC, bool WIN>
__device__ __forceinline__ void trace_col(const FillArgs& a, const PairDesc& pd, unsigned char* obuf, unsigned* pfl,
                                          int lane, int sb, int& o_len, int2& o_end, bool& o_out) {
  const int nblk = pd.bits_nblk, win = WIN ? pd.bits_w : 0;
  const int64_t bdw = (int64_t)nblk * 1024;  // dwords per band
  const unsigned* mat = a.mat + pd.mat_off;
  const bool segd = pd.spec_every > 0;
  // segments (nwk_internal.h colseg_*): band b's records at recs + rec_off + b
  // 2048, info at seginfo + 4 (seg_off + b), moves at segops + segops_off + b cap
  u64* const srec = a.recs + pd.rec_off;
  int* const sinfo = a.seginfo + 4 * pd.seg_off;
  uint8_t* const smov = a.segops + pd.segops_off;
  const int64_t scap = colseg_cap(pd.n);
  const u64 ep20 = (u64)(a.epoch & 0xfffffu);
  uint8_t* ops = SPEC                ? smov + (int64_t)sb * scap
                 : a.ops_host ? a.ops_host + (pd.ops_off - a.ops_base)  // (streamed host finalize)
                              : a.ops + pd.ops_off;
  const unsigned ob = (unsigned)(uintptr_t)obuf;
  int Lc = 0, flushed = 0;
  auto flush = [&](int upto) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int from = flushed & ~3;
    for (int o = from + 4 * lane; o < upto; o += 256) {
      unsigned v;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(ob + (unsigned)(o & (kTraceRing - 1)))
                   : "memory");
      *reinterpret_cast<unsigned*>(ops + o) = v;
    }
    flushed = upto;
  };
  // (pair walk) append n moves from src (a finished segment) to ops at Lc:
  // head bytes to a dword boundary, dwords (two aligned source dwords and
  // v_alignbyte each), tail bytes; the ring gets the bytes of the last partial
  // dword, which the next flush rewrites
  auto seg_copy = [&](const uint8_t* src, int n) {
    flush(Lc);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int d0 = Lc;
    const int h = smin(n, (4 - (d0 & 3)) & 3);
    if (lane < h) ops[d0 + lane] = src[lane];
    const int nd = (n - h) >> 2;
    const uintptr_t sa = (uintptr_t)(src + h);
    const unsigned* s0 = reinterpret_cast<const unsigned*>(sa & ~(uintptr_t)3);
    const unsigned sh = (unsigned)(sa & 3);
    unsigned* dw = reinterpret_cast<unsigned*>(ops + d0 + h);
    for (int w0 = 0; w0 < nd; w0 += 256) {
      unsigned lo[4], hi[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int w = w0 + 64 * k + lane;
        lo[k] = w < nd ? s0[w] : 0u;
        hi[k] = w < nd ? s0[w + 1] : 0u;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int w = w0 + 64 * k + lane;
        if (w < nd) dw[w] = __builtin_amdgcn_alignbyte(hi[k], lo[k], sh);
      }
    }
    const int t = (n - h) & 3;
    if (lane < t) ops[d0 + h + 4 * nd + lane] = src[h + 4 * nd + lane];
    const int e = d0 + n, e0 = e & ~3;
    if (lane < e - e0 && e0 + lane >= d0)
      asm volatile("ds_write_b8 %0, %1" ::"v"(ob + (unsigned)((e0 + lane) & (kTraceRing - 1))), "v"((unsigned)src[e0 + lane - d0])
                   : "memory");
    Lc = e;
    flushed = e;
  };
  int b = (pd.m - 1) / kBR, r = (pd.m - 1) % kBR, c = pd.n - 1;
  if (!SPEC && a.dbg_corrupt == pd.slot + 1) {
    // (tests of the fill-vs-walk guard) flip the stored D bit of cell (m, n):
    // lane r / 32 holds it at step c + r / 32, bit r % 32 of the diag word
    const int s = c + (r >> 5), rel = (s >> 3) - bits_blk_lo(b, pd.m, pd.n, win);
    if (lane == 0 && (unsigned)rel < (unsigned)nblk)
      __hip_atomic_fetch_xor((gu32*)(mat + (int64_t)b * bdw + (int64_t)rel * 1024 + ((s & 7) >> 2) * 256 + 4 * (r >> 5) + (s & 3)),
                             1u << (r & 31), BITS_RLX);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if constexpr (SPEC) {  // band sb's last row, at the proportional diagonal's column
    b = sb;
    r = kBR - 1;
    c = (int)(((int64_t)(sb + 1) * kBR - 1) * pd.n / pd.m);
    c = c > pd.n - 1 ? pd.n - 1 : c;
  }
  if (a.dbg_notrace) c = -1;  // NWK_NOTRACE (fill timing): no moves
  int tb = -1, blo = 0, slo = 0;
  const int64_t lim = (int64_t)win * pd.m;
  if (win > 0 && c >= 0) {  // the walk's first cell
    const int64_t dev = (int64_t)c * pd.m - ((int64_t)b * kBR + r) * pd.n;
    if (dev > lim || dev < -lim) c = -2;  // (out below)
  }
  if (SPEC && c >= 0 && lane == 0)  // the segment's first cell: row kBR - 1, move 0
    __hip_atomic_store(srec + (int64_t)sb * kBR + kBR - 1, (ep20 << 44) | ((u64)c << 22), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  bool bad = false, out = false;
  int nomerge = -1;  // a band whose segment failed
  unsigned n_merge = 0;
  // The current tile (cts, tta: columns cts - 63 .. cts, row-lanes tta - 3 ..
  // tta of band ctb) stays while the walk is inside it -- a pass that runs off
  // its key window only re-windows -- and one tile ahead is in flight: where
  // the walk is predicted to leave the current one (rows per column ~ m / n),
  // through its left edge (64 columns on, 24 rows of slack above the entry
  // row) or its top (the row-lanes above, 16 columns of slack to the right).
  unsigned vd[4] = {0, 0, 0, 0}, vu[4] = {0, 0, 0, 0};
  int cts = -1, tta = -1, ctb = -1, ncts = -1, nta = -1, nb_ = -1;
  // (pair walk) band bb's segment records of the tile's 128 rows, two per lane
  u64 rq[2] = {0, 0}, nrq[2] = {0, 0};
  auto recs_on = [&](int bb) { return !SPEC && segd && bb < pd.nbands - 1 && bb != nomerge; };
  auto load_recs = [&](int bb, int ta_, u64 (&q)[2]) {
    const int row = (ta_ > 3 ? 32 * (ta_ - 3) : 0) + 2 * lane;
    const u64* p = srec + (int64_t)bb * kBR + row;
    q[0] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    q[1] = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  auto load_tile = [&](int bb, int blo_, int cts_, int ta_, unsigned (&d)[4], unsigned (&u)[4]) {
    const int cl = cts_ - lane;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = ta_ - k < 0 ? 0 : ta_ - k;
      int step = cl + t;
      int rel = (step >> 3) - blo_;
      const bool okl = cl >= 0 && (unsigned)rel < (unsigned)nblk;
      step = okl ? step : 0;
      rel = okl ? rel : 0;
      const unsigned* p = mat + (int64_t)bb * bdw + (int64_t)rel * 1024 + ((step & 7) >> 2) * 256 + 4 * t + (step & 3);
      d[k] = __builtin_nontemporal_load(p);
      u[k] = __builtin_nontemporal_load(p + 512);
    }
  };
  // the tile ahead goes to LDS (pfl: 8 x 64 dwords per wave, d[k] at k * 64,
  // u[k] at (4 + k) * 64) by LDS-DMA loads: no VGPR is the destination of a
  // load in flight, so the compiler never waits on it inside the walk (with
  // register destinations it did, for an undefined phi input it materialized
  // from the first load's register)
  const unsigned pfb = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)pfl);
  auto prefetch_lds = [&](int bb, int blo_, int cts_, int ta_) {
    const int cl = cts_ - lane;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = ta_ - k < 0 ? 0 : ta_ - k;
      int step = cl + t;
      int rel = (step >> 3) - blo_;
      const bool okl = cl >= 0 && (unsigned)rel < (unsigned)nblk;
      step = okl ? step : 0;
      rel = okl ? rel : 0;
      const unsigned* p = mat + (int64_t)bb * bdw + (int64_t)rel * 1024 + ((step & 7) >> 2) * 256 + 4 * t + (step & 3);
      asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(p), "s"(__builtin_amdgcn_readfirstlane(pfb + 256u * k))
                   : "memory", "m0");
      asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(p + 512), "s"(__builtin_amdgcn_readfirstlane(pfb + 256u * (4 + k)))
                   : "memory", "m0");
    }
  };
  auto rowlo_of = [](int ta_) { return ta_ > 3 ? 32 * (ta_ - 3) : 0; };
  const int64_t rpc = ((int64_t)pd.m << 16) / pd.n;  // rows per column (16.16)
  const int64_t cpr = ((int64_t)pd.n << 16) / pd.m;  // columns per row (16.16; no 64-bit divide per tile)
  // key window base below the entry key: wide pairs' walks climb keys (L
  // moves, +1), tall pairs' descend (U moves, -1)
  const int kback = rpc < 52429 ? 4 : (rpc > 81920 ? 28 : 16);
  const u64 tc0 = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
  unsigned n_tiles = 0, n_dem = 0, n_stops = 0;
#if NWK_TRACE_PROF  // (A/B build: cycles per phase, printed per pair)
  u64 p_sw = 0, p_wait = 0, p_win = 0, p_walk = 0, p_out = 0, n_pass = 0;
#endif
  if (c == -2) out = true;
  while (!out && c >= 0 && (b > 0 || r >= 0)) {
    if (r < 0) {  // into the band above
      if constexpr (SPEC) break;  // (a segment ends at its band's top)
      --b;
      r += kBR;
    }
    if (b != tb) {
      blo = __builtin_amdgcn_readfirstlane(bits_blk_lo(b, pd.m, pd.n, win));
      slo = 8 * blo;
      tb = b;
    }
    const int ta = r >> 5;
    {
      const int step = c + ta;
      if ((unsigned)((step >> 3) - blo) >= (unsigned)nblk || c < slo) {  // the path left the stored window
        out = true;
        break;
      }
    }
#if NWK_TRACE_PROF
    const u64 pt0 = __builtin_amdgcn_s_memtime();
#endif
    if (Lc - flushed >= kTraceRing - 256) flush(Lc & ~3);  // (a pass adds <= 64 + 128 moves)
    if (!(ctb == b && c > cts - 64 && ta <= tta && r >= rowlo_of(tta))) {
      if (nb_ == b && c <= ncts && c > ncts - 64 && ta <= nta && r >= rowlo_of(nta)) {  // the tile ahead
#if NWK_TRACE_PROF
        const u64 pw0 = __builtin_amdgcn_s_memtime();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        p_wait += __builtin_amdgcn_s_memtime() - pw0;
#endif
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the LDS-DMA loads)
        cts = ncts;
        tta = nta;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          vd[k] = pfl[64 * k + lane];
          vu[k] = pfl[64 * (4 + k) + lane];
        }
        rq[0] = nrq[0];
        rq[1] = nrq[1];
      } else {
        ++n_dem;
        cts = c;
        tta = ta;
        load_tile(b, blo, cts, tta, vd, vu);
        if (recs_on(b)) load_recs(b, tta, rq);
        __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
      }
      ctb = b;
      ++n_tiles;
      // the tile after this one
      const int tlo = rowlo_of(tta);
      const int64_t cl = c - (cts - 64);          // columns to the left edge
      const int64_t rt = r - tlo + 1;             // rows to the top
      nb_ = -1;
      if (tlo > 0 && (rt << 16) < cl * rpc) {     // leaves through the top
        const int ce = c - (int)((rt * cpr) >> 16);
        const int c2 = smin(cts, ce + 16);
        if (c2 >= slo) {
          nb_ = b;
          ncts = __builtin_amdgcn_readfirstlane(c2);
          nta = __builtin_amdgcn_readfirstlane((tlo >> 5) - 1);
        }
      } else {                                    // through the left edge
        const int c2 = cts - 64;
        const int rp = r - (int)((cl * rpc) >> 16);
        if (c2 >= slo && rp >= 0) {
          nb_ = b;
          ncts = c2;
          int pa = (rp + 24) >> 5;
          pa = pa > kBR / 32 - 1 ? kBR / 32 - 1 : pa;
          nta = __builtin_amdgcn_readfirstlane(pa);
        }
      }
      if (nb_ >= 0) {
        prefetch_lds(b, blo, ncts, nta);
        if (recs_on(b)) load_recs(b, nta, nrq);
      }
    }
    const int trowlo = rowlo_of(tta);
    // (pair walk) is this cell on band b's segment?  Row r's record: the entry
    // column c_hi and move index k; row r - 1's index gives the row's L moves,
    // so its cells are c_hi - nL .. c_hi
    if (recs_on(b)) {
      const int ix = r - trowlo;  // 0 .. 127
      auto rec_at = [&](int x) {
        const u64 v = (x & 1) ? rq[1] : rq[0];
        const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, x >> 1);
        const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), x >> 1);
        return ((u64)hi << 32) | lo;
      };
      const u64 e = rec_at(ix);
      int kk = -1;
      if ((e >> 44) == ep20) {
        const int chi = (int)((e >> 22) & 0x3fffffu), khi = (int)(e & 0x3fffffu);
        if (c == chi) {
          kk = khi;
        } else if (c < chi && ix > 0) {
          const u64 e1 = rec_at(ix - 1);
          if ((e1 >> 44) == ep20 && c >= chi - ((int)(e1 & 0x3fffffu) - khi - 1)) kk = khi + (chi - c);
        }
      }
      if (kk >= 0) {
        // merged: wait for the segment to finish, then its moves kk .. len - 1
        int* inf = sinfo + 4 * b;
        for (;;) {
          const unsigned f = __builtin_amdgcn_readfirstlane(__hip_atomic_load((gu32*)inf, BITS_RLX));
          if (f == a.epoch) break;
          if (__builtin_amdgcn_readfirstlane(__hip_atomic_load((gu32*)a.err, BITS_RLX)) != 0u) {
            bad = true;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        if (bad) break;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        const int slen = __builtin_amdgcn_readfirstlane(__hip_atomic_load(inf + 1, BITS_RLX));
        const int xi = __builtin_amdgcn_readfirstlane(__hip_atomic_load(inf + 2, BITS_RLX));
        const int xc = __builtin_amdgcn_readfirstlane(__hip_atomic_load(inf + 3, BITS_RLX));
        if (slen < 0 || kk > slen) {
          nomerge = b;  // (failed segment: walk the band)
        } else {
          seg_copy(smov + (int64_t)b * scap + kk, slen - kk);
          ++n_merge;
          b = xi >= 0 ? xi / kBR : -1;
          r = xi - b * kBR;
          if (xi < 0) {  // the segment reached row -1 (band 0's top)
            b = 0;
            r = -1;
          }
          c = xc;
          if (Lc > pd.m + pd.n) {
            bad = true;
            break;
          }
          continue;
        }
      }
    }
#if NWK_TRACE_PROF
    const u64 pt1 = __builtin_amdgcn_s_memtime();
    p_sw += pt1 - pt0;
#endif
    const int LL = smin(63, cts - slo);  // last lane whose column is >= the lowest stored step
    int L = cts - c;
    int K = r + L;
    // windowed storage keeps only the lane words holding a cell within bits_w
    // columns of the diagonal: a cell read must have |dev| <= lim, dev = c m - i n.
    // Tiles wholly inside skip the checks; near the window's edge each run's end
    // cells are checked (dev is linear along a D or U run)
    const int64_t ib = (int64_t)b * kBR;
    const bool wchk = WIN && win > 0 && ((int64_t)cts * pd.m - (ib + trowlo) * pd.n > lim ||
                                  (int64_t)(cts - 63) * pd.m - (ib + trowlo + 127) * pd.n < -lim);
    auto outside = [&](int Ll, int Kk) {
      const int64_t dev = (int64_t)(cts - Ll) * pd.m - (ib + Kk - Ll) * pd.n;
      return dev > lim || dev < -lim;
    };
    const int Kb = K - kback;
    // key window: lane l's bit i = its cell at row Kb + i - l: bit q of the
    // column {0, vd[3], vd[2], vd[1], vd[0], 0} (rows below / above the tile read 0)
    unsigned WD, WU;
    {
      const int q = Kb - lane - 32 * (tta - 3) + 32;
      const int dq = q >> 5, sh = q & 31;
      const bool ok = q >= 0 && q < 160;
      const unsigned dlo = dq == 1 ? vd[3] : dq == 2 ? vd[2] : dq == 3 ? vd[1] : dq == 4 ? vd[0] : 0u;
      const unsigned dhi = dq == 0 ? vd[3] : dq == 1 ? vd[2] : dq == 2 ? vd[1] : dq == 3 ? vd[0] : 0u;
      const unsigned ulo = dq == 1 ? vu[3] : dq == 2 ? vu[2] : dq == 3 ? vu[1] : dq == 4 ? vu[0] : ~0u;
      const unsigned uhi = dq == 0 ? vu[3] : dq == 1 ? vu[2] : dq == 2 ? vu[1] : dq == 3 ? vu[0] : ~0u;
      WD = ok ? __builtin_amdgcn_alignbit(dhi, dlo, sh) : 0u;
      WU = ok ? __builtin_amdgcn_alignbit(uhi, ulo, sh) : ~0u;  // stored up word: 0 = UP
    }
    const unsigned WL = WU & ~WD;  // cells that move L: neither D nor U
#if NWK_TRACE_PROF
    const u64 pt2 = __builtin_amdgcn_s_memtime();
    p_win += pt2 - pt1;
#endif
    const int L0 = L;
    u64 finL = 0;          // lanes whose last move is L
    unsigned nUv = 0;      // per lane: U moves (written by v_writelane)
    int maxU = 0;
    // a horizontal run: after an L move the walk stays on row rr = K - L; one
    // ballot of the row's cells (lane l's key-window bit rr - Kb + l) that move
    // L takes the whole run to the first lane that moves D or U (or to the edge
    // of the readable cells) -- wide pairs' paths are mostly long L runs
    // (big13 35k x 90k: 55k L moves of 90k), one loop trip each before.
    // False: the run's last cell is outside the stored window.
    auto lrun = [&](auto chk_t) -> bool {
      constexpr bool CHK = decltype(chk_t)::value;
      const int rr = K - L;
      const int lend_r = smin(LL, 31 + Kb - rr) + 1;  // first lane whose row-rr cell is not readable
      if (L >= lend_r) return true;
      // (lanes whose bit rr - Kb + l is off the window are past lend_r: v_bfe's
      // offset wraps there, and the min below discards them)
      const u64 Lm = __builtin_amdgcn_ballot_w64(__builtin_amdgcn_ubfe(WL, (unsigned)(rr - Kb + lane), 1u) != 0u);
      const int le = sminu(sff1u(~Lm & (~0ull << L)), lend_r);
      if (le == L) return true;
      if constexpr (CHK) {
        if (outside(le - 1, rr + le - 1)) return false;
      }
      finL |= (le >= 64 ? ~0ull : ((1ull << le) - 1ull)) & (~0ull << L);
      L = le;
      K = rr + le;
      return true;
    };
    // The run loop, all scalar; the CHK copy checks the stored lane words
    // (windowed storage, only in tiles near the window's edge).
    auto walk = [&](auto chk_t) {
      constexpr bool CHK = decltype(chk_t)::value;
      for (;;) {
        const int bnd = smin(K - trowlo, LL);
        if (L > bnd) break;  // the cell is below the tile's rows or past its columns
        const int i = K - Kb;
        if ((unsigned)i > 31u) break;  // off the key window: re-window
        if constexpr (CHK) {
          if (outside(L, K)) {
            out = true;
            break;
          }
        }
        // (every stop changes the key: the key's lane masks are built each trip)
        const u64 Dm = __builtin_amdgcn_ballot_w64(__builtin_amdgcn_ubfe(WD, (unsigned)i, 1u) != 0u);
        const u64 Um = __builtin_amdgcn_ballot_w64(__builtin_amdgcn_ubfe(WU, (unsigned)i, 1u) == 0u);
        const int lend = bnd + 1;  // first lane past the readable cells of this key
        const u64 stops = ~Dm & (~0ull << L);
        const int ls = sminu(sff1u(stops), lend);  // (no stop: ff1 = -1)
        if constexpr (CHK) {
          if (outside(ls < lend ? ls : lend - 1, K)) {  // the run's last cell read
            out = true;
            break;
          }
        }
        if (ls >= lend) {  // D moves through lanes L .. lend - 1
          L = lend;
          break;
        }
        if ((Um >> ls) & 1ull) {
          // a U move, then down lane ls's column: U while D is clear and U set
          const unsigned wd = (unsigned)__builtin_amdgcn_readlane((int)WD, ls);
          const unsigned wu = (unsigned)__builtin_amdgcn_readlane((int)WU, ls);
          const int jlo = smax(trowlo + ls - Kb, 0);  // lowest key bit inside the tile's rows
          const unsigned below = i >= 31 ? ~0u : ((2u << i) - 1u);
          const unsigned stopm = (wd | wu) & below & ~((1u << jlo) - 1u);
          if constexpr (CHK) {
            if (outside(ls, Kb + (stopm ? 31 - __builtin_clz(stopm) : jlo))) {  // the vertical run's last cell
              out = true;
              break;
            }
          }
          if (stopm == 0u) {  // the run leaves the tile's rows (or the key window): U moves down to there
            const int nU = i - jlo + 1;
            nUv = writelane(nUv, nU, ls);
            maxU = nU > maxU ? nU : maxU;
            L = ls;
            K = Kb + jlo - 1;
            break;
          }
          const int j = 31 - __builtin_clz(stopm);
          const int nU = i - j;
          nUv = writelane(nUv, nU, ls);
          maxU = nU > maxU ? nU : maxU;
          L = ls + 1;
          if ((wd >> j) & 1u) {  // the cell at key j moves D
            K = Kb + j;
            continue;
          }
          finL |= 1ull << ls;  // ... or L
          K = Kb + j + 1;
        } else {  // an L move
          finL |= 1ull << ls;
          L = ls + 1;
          K = K + 1;
        }
        if (!lrun(chk_t)) {
          out = true;
          break;
        }
      }
    };
    // (K and L pinned in SGPRs across the branch: an undefined phi input for
    // them was materialized as v_readfirstlane of the next tile's load
    // register, and the wait for that load then sat on every pass)
    asm volatile("" : "+s"(K), "+s"(L));
    // (the asm walk's operands: copies defined, and used, on both paths)
    int Ka = K, La = L, mU = maxU;
    u64 fL = finL;
    if (WIN && wchk) {
      asm volatile("" ::"s"(Ka), "s"(La), "s"(mU), "s"(fL));
      if constexpr (WIN) walk(std::true_type{});
      asm volatile("" : "+s"(K), "+s"(L));
    } else {
#if NWK_COL_CWALK  // (A/B: the compiled walk)
      walk(std::false_type{});
#else
      unsigned nv = nUv;
      walk_asm(WD, WU, WL, lane, Kb, trowlo, LL, Ka, La, fL, nv, mU);
      K = Ka;
      L = La;
      finL = fL;
      nUv = nv;
      maxU = mU;
#endif
    }
#if NWK_TRACE_PROF
    const u64 pt3 = __builtin_amdgcn_s_memtime();
    p_walk += pt3 - pt2;
    ++n_pass;
#endif
    // the tile's moves in walk order: lanes L0 .. L - 1 are done (U^nU, then D
    // or L), lane L (when <= 63) holds only its U moves so far
    {
      const bool vis = lane >= L0 && lane <= L;
      const bool fin = lane >= L0 && lane < L;
      const unsigned nU = vis ? nUv : 0u;
      const unsigned cnt = nU + (fin ? 1u : 0u);
      const unsigned inc = shadev::wave_incl_scan(cnt, lane);
      const unsigned off = inc - cnt;
      const unsigned tot = (unsigned)__builtin_amdgcn_readlane((int)inc, 63);
      for (int j = 0; j < maxU; ++j)
        if ((unsigned)j < nU)
          asm volatile("ds_write_b8 %0, %1" ::"v"(ob + (unsigned)((Lc + (int)off + j) & (kTraceRing - 1))), "v"((unsigned)'U')
                       : "memory");
      if (fin) {
        const unsigned ch = ((finL >> lane) & 1ull) ? 'L' : 'D';
        asm volatile("ds_write_b8 %0, %1" ::"v"(ob + (unsigned)((Lc + (int)(off + nU)) & (kTraceRing - 1))), "v"(ch)
                     : "memory");
      }
      if constexpr (SPEC) {
        // the rows this pass entered: lane l's U moves enter rows r0 - 1 .. r0 - nU
        // at its column, its D move row r0 - nU - 1 at the next; r0 = the pass's
        // row minus the rows of the lanes before (exclusive scan of nU + D)
        const bool isD = fin && !((finL >> lane) & 1ull);
        const unsigned dr = nU + (isD ? 1u : 0u);
        const int r0 = r - (int)(shadev::wave_incl_scan(dr, lane) - dr);
        const int col = cts - lane;
        u64* rb = srec + (int64_t)sb * kBR;
        for (int j = 1; j <= maxU + 1; ++j) {
          const bool u = (unsigned)j <= nU, d = isD && (unsigned)j == nU + 1;
          const int rr = r0 - j;
          if ((u || d) && rr >= 0) {
            const int cc = d ? col - 1 : col;
            const u64 k = (u64)(Lc + (int)off + j);
            if (cc >= 0)
              __hip_atomic_store(rb + rr, (ep20 << 44) | ((u64)cc << 22) | k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      }
      Lc += (int)tot;
      if (a.stamps) n_stops += (unsigned)__builtin_popcountll(__builtin_amdgcn_ballot_w64(fin && ((finL >> lane) & 1ull || nU)));
    }
    r = K - L;
    c = cts - L;
#if NWK_TRACE_PROF
    p_out += __builtin_amdgcn_s_memtime() - pt3;
#endif
    if (Lc > pd.m + pd.n) {
      bad = true;
      break;
    }
  }
  if constexpr (SPEC) {
    // the segment: its moves, then {length (-1: failed), exit cell} and the flag
    flush(Lc);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) {
      int* inf = sinfo + 4 * sb;
      __hip_atomic_store(inf + 1, (out || bad) ? -1 : Lc, BITS_RLX);
      __hip_atomic_store(inf + 2, b * kBR + r, BITS_RLX);
      __hip_atomic_store(inf + 3, c, BITS_RLX);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (lane == 0) __hip_atomic_store((gu32*)(sinfo + 4 * sb), a.epoch, BITS_RLX);
    return;
  }
  if (a.dbg_badwalk == pd.slot + 1) bad = true;  // (tests: a failed walk must never reach the host as a result)
  if (bad && lane == 0) atomicOr(a.err, 16u);
  if (a.stamps && lane == 0) {
    u64* x = a.stamps + 8 * pd.slot;
    x[2] = __builtin_amdgcn_s_memtime() - tc0;
    x[3] = n_stops;
    x[4] = (u64)Lc;
    x[5] = ((u64)n_tiles << 32) | ((u64)n_dem << 16) | (u64)(n_merge & 0xffffu);
  }
  flush(Lc);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if NWK_TRACE_PROF
  if (lane == 0)
    printf("trace_col %d x %d: moves %d passes %llu tiles %u demand %u | cycles switch %llu (wait %llu) window %llu walk %llu out %llu\n",
           pd.m, pd.n, Lc, (unsigned long long)n_pass, n_tiles, n_dem, (unsigned long long)p_sw, (unsigned long long)p_wait,
           (unsigned long long)p_win, (unsigned long long)p_walk, (unsigned long long)p_out);
#endif
  o_len = out ? 0 : Lc;
  o_end = (a.dbg_notrace || out) ? make_int2(pd.m, pd.n) : make_int2(b * kBR + r + 1, c + 1);
  o_out = out;
  if (lane == 0) {
    a.oplen[pd.slot] = o_len;
    a.endij[pd.slot] = o_end;
    if (out) a.retry[pd.slot] = 1;
    if (a.host_rec) {
      int* h = a.host_rec + kHostRecInts * pd.slot;
      h[1] = out ? -1 : bad ? -2 : o_len;  // -1: re-run wider, -2: failed (never finalized)
      h[2] = o_end.x;
      h[3] = o_end.y;
      h[4] = a.endv ? (int)__hip_atomic_load((gu32*)(a.endv + pd.slot), BITS_RLX) : 0;  // the fill's H(m, n)
    }
  }
  if (a.host_rec) {  // the moves (host memory) and the record, then its flag
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __threadfence_system();
    if (lane == 0)
      __hip_atomic_store(a.host_rec + kHostRecInts * pd.slot, (int)a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Waves per SIMD the kernel is compiled for (register budget 512 / WPE): the
// fused-finalize instantiation at NWK_COL_WPE (4); the plain one at 4 or, for
// jobs of a few rounds of bands (launch_col's wpe), NWK_COL_WPE_HI (5, <= 96
// VGPRs, a few spills outside the step loop): C3's 4-rank shard (3.1 rounds of
// 4,096 slots) 60.5 -> 48.6 ms, the 8-rank one 32.2 -> 30.5 ms, big13 equal;
// the streamed fused ranks (C4 W = 8) are faster at 4 (22.0 vs 24.5 ms)
// (profiles/r05/ab/col_wpe.txt).
#ifndef NWK_COL_WPE
#define NWK_COL_WPE 4
#endif
#ifndef NWK_COL_WPE_HI
#define NWK_COL_WPE_HI 5
#endif

// FUSE: the instantiation with the fused finalize (FillArgs::fuse_fin)
template <int NP, int SR, bool FUSE, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void nw_align_col(FillArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char obuf_all[4][kTraceRing];
  __shared__ __attribute__((aligned(16))) unsigned pf_all[4][512];  // trace_col's tile ahead (LDS-DMA)
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  unsigned* prog = a.prog ? a.prog + blockIdx.x * 4 + wid : nullptr;  // NWK_WATCHDOG markers
  // verbose >= 2 timeline (FillArgs::stamps, layout in nwk_runtime.cpp)
  if (a.stamps && threadIdx.x == 0) atomicMin(a.stamps + 11 * a.ntasks_pairs, (u64)__builtin_amdgcn_s_memrealtime());

  for (;;) {
    if constexpr (FUSE) {  // queued pairs to hash: whole groups between fill tasks
      while (hq_hash(a, lane, false)) {
      }
    }
    unsigned tk = 0;
    if (lane == 0) tk = atomicAdd(a.counter, 1u);
    tk = __builtin_amdgcn_readfirstlane(tk);
    BITS_PROG(0x10000000u | tk);
    if (tk >= (unsigned)a.ntasks) {
      if constexpr (FUSE) hq_drain(a, lane);
      BITS_PROG(0x60000000u);
      return;
    }
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load((gu32*)a.err, BITS_RLX)) != 0u) return;
    const u64 t_task = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
    const int2 task = a.tasks[tk];
    const PairDesc pd = a.pairs[task.x];
    const int band = task.y;
    const int R0 = band * kBR;
    // the longest spans of a span-bound batch issue ahead of the other fill waves
    // (band_prio: a pair's bands run as a pipeline at the pace of its slowest
    // upstream band, so the upper bands issue first -- 3 .. 0 by quarter of the pair)
    const int bprio = a.band_prio ? 3 - (4 * band) / pd.nbands : 0;
    const int prio = pd.prio > bprio ? pd.prio : bprio;
    if (prio >= 3) __builtin_amdgcn_s_setprio(3);
    else if (prio == 2) __builtin_amdgcn_s_setprio(2);
    else if (prio == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
    // code bit planes of rows R0 + 32 lane + b (rows past m: code 0, never traced)
    unsigned x0 = 0, x1 = 0;
    {
      const int base = R0 + 32 * lane;
      const int nv = pd.m - base;
      const uint8_t* xc = a.codes + pd.x_off + base;
#pragma unroll
      for (int b = 0; b < 32; ++b) {
        const unsigned cd = b < nv ? (unsigned)xc[b] : 0u;
        x0 |= (cd & 1u) << b;
        x1 |= ((cd >> 1) & 1u) << b;
      }
    }
    unsigned l[NP], acc[NP], pub[NP];
    u64 c[NP], inj[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      l[k] = acc[k] = pub[k] = 0u;
      c[k] = inj[k] = 0ull;
    }
    const bool from_above = band > 0;
    const bool to_below = band + 1 < pd.nbands;
    const int nw = (pd.n + 31) >> 5;  // 32-column words of a row
    const int nsb = pd.sblocks;
    const u64* gin = reinterpret_cast<const u64*>(a.bnd) + pd.bnd_off + (int64_t)(from_above ? band - 1 : 0) * nw * NP;
    u64* gout = a.bnd + pd.bnd_off + (int64_t)band * nw * NP;
    const int nblk = pd.bits_nblk, blo = bits_blk_lo(band, pd.m, pd.n, pd.bits_w);
    unsigned* mb = a.mat + pd.mat_off + (int64_t)band * nblk * 1024 + lane * 4;
    // windowed storage, per lane and 8-step block: its words hold rows R0 + 32 lane ..
    // + 31 at columns s0 - lane .. + 7, so dev = c m - i n spans [hi - 7 m - 31 n, hi]
    // with hi = (s0 - lane + 7) m - (R0 + 32 lane) n = s0 m + hi0 (bits_lane_stored)
    const bool win = pd.bits_w > 0;
    const int64_t lim = (int64_t)pd.bits_w * pd.m, hlim = lim + 7ll * pd.m + 31ll * pd.n;
    const int64_t hi0 = (int64_t)(7 - lane) * pd.m - (int64_t)(R0 + 32 * lane) * pd.n;
    // y windows: lane t's window for the half starting at step s_h is position s_h - t
    const unsigned* ywp = a.yw + 2 * (pd.e_off - (int64_t)lane);
    unsigned wc0 = ywp[0], wc1 = ywp[1];
    // granule k of a 32-column word is polled by lane k; every lane loads one
    // (lanes >= NP a copy) so no branch depends on the lane: a lane-dependent
    // branch here would make the compiler treat the carries as per-lane values
    const bool gl = lane < NP;
    const int gk = lane & (NP - 1);
    u64 g = 0;
    if (from_above) g = __hip_atomic_load((gu64*)(gin + gk), BITS_RLX);
    bool ok = true;
    u64 cyc_wait = 0, cyc_wait0 = 0, n_wait = 0;  // (verbose >= 2 timeline)
    // fill-vs-walk guard: G(m, n) = -sum of v down column n (G-space borders are
    // 0), so each band adds minus the vertical differences of its rows < m at
    // column n - 1 (0-based), taken by lane t at step n - 1 + t: the steps of
    // super-blocks sbe .. nsb - 1 only
    const int capc = pd.n - 1;
    const bool want_end = a.endv != nullptr;
    const int sbe = want_end ? (capc >> 6 > 1 ? capc >> 6 : 1) : nsb;
    const int capx = want_end ? capc : -1000;
    int cnt = 0;                  // (uniform)
    const int nvr0 = pd.m - R0;   // rows < m from lane 0's first row on

    auto half = [&](int h, auto mask_t, auto end_t) {
      constexpr bool MASK = decltype(mask_t)::value;
      constexpr bool END = decltype(end_t)::value;
      const unsigned* wp = ywp + 64 * (h + 1);
      const unsigned nx0 = wp[0], nx1 = wp[1];  // the next half's window
      if (from_above) {
        if (h < nw) {
          if (!wall(!gl || (unsigned)(g >> 32) == a.epoch)) {
            const u64 tw = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
            g = bits_wait(gin + (int64_t)h * NP + gk, gl, a.epoch, g, a.err);
            if (a.stamps) {
              const u64 d = __builtin_amdgcn_s_memtime() - tw;
              cyc_wait += d;
              if (h == 0) cyc_wait0 = d;
              ++n_wait;
            }
            // (a failed wait ends the task after this half, which publishes nothing; the
            // error word fails the call.  No early return: it would leave the carries
            // undefined on one path, and the compiler then moves them out of SGPRs)
            if (!wall(!gl || (unsigned)(g >> 32) == a.epoch)) ok = false;
          }
          const unsigned dat = (unsigned)g;
#pragma unroll
          for (int k = 0; k < NP; ++k) inj[k] = (u64)(unsigned)__builtin_amdgcn_readlane((int)dat, k);
          if (h + 1 < nw) g = __hip_atomic_load((gu64*)(gin + (int64_t)(h + 1) * NP + gk), BITS_RLX);
        } else {
#pragma unroll
          for (int k = 0; k < NP; ++k) inj[k] = 0ull;
        }
      }
      auto blk = [&](auto bc) {
        constexpr int B = decltype(bc)::value;
        const int s0 = 32 * h + 8 * B;
        const int rel = (s0 >> 3) - blo;
        // stored: the block is among the band's stored steps and (windowed) this
        // lane's words of it hold a cell within bits_w columns of the diagonal
        const bool sto = (unsigned)rel < (unsigned)nblk && (!win || bits_lane_stored(hi0 + (int64_t)s0 * pd.m, lim, hlim));
        unsigned* st = mb + (int64_t)rel * 1024;
        col_block<NP, SR, MASK, B == 3, B, END>(s0, lane, x0, x1, wc0, wc1, l, c, acc, inj, pub, st, sto, capx, nvr0,
                                                cnt);
      };
      blk(std::integral_constant<int, 0>{});
      blk(std::integral_constant<int, 1>{});
      blk(std::integral_constant<int, 2>{});
      blk(std::integral_constant<int, 3>{});
      // publish the band's last row, columns 32 (h - 2) .. + 31 (lane 63's carries of steps 32 h - 1 .. 32 h + 30,
      // MSB first in pub)
      if (to_below && ok && h >= 2 && h - 2 < nw) {
        unsigned v = 0;
#pragma unroll
        for (int k = 0; k < NP; ++k) v = gk == k ? __builtin_bitreverse32(pub[k]) : v;
        // (every lane stores: lanes >= NP repeat lane gk's granule, so no branch depends on the lane)
        __hip_atomic_store((gu64*)(gout + (int64_t)(h - 2) * NP + gk), ((u64)a.epoch << 32) | v, BITS_RLX);
      }
      wc0 = nx0;
      wc1 = nx1;
    };
    // the first super-block (columns < 0 masked) peeled off the loop; the last
    // ones (column n - 1) take the guard's end value
    // (always the END form: an if / else around the peeled halves makes the
    // compiler treat the SGPR carries as divergent; capx = -1000 matches nothing)
    half(0, std::true_type{}, std::true_type{});
    half(1, std::true_type{}, std::true_type{});
    int sb = 1;
    for (; sb < sbe && ok; ++sb) {
      half(2 * sb, std::false_type{}, std::false_type{});
      half(2 * sb + 1, std::false_type{}, std::false_type{});
    }
    for (; sb < nsb && ok; ++sb) {
      half(2 * sb, std::false_type{}, std::true_type{});
      half(2 * sb + 1, std::false_type{}, std::true_type{});
    }
    BITS_PROG(0x30000000u);
    if (!ok) return;
    if (want_end) {  // this band's part of H(m, n): - sum v (+ (m + n) pgap once, band 0)
      if (lane == 0)
        __hip_atomic_fetch_add((gu32*)(a.endv + pd.slot), (unsigned)(band == 0 ? (pd.m + pd.n) * a.pgap - cnt : -cnt),
                               BITS_RLX);
    }
    if (a.stamps && lane == 0) {  // per pair: band cycles
      atomicAdd(a.stamps + 8 * pd.slot + 6, (u64)(__builtin_amdgcn_s_memtime() - t_task));
      atomicAdd(a.stamps + 8 * pd.slot + 7, cyc_wait);
      atomicAdd(a.stamps + 8 * a.ntasks_pairs + 3 * pd.slot, cyc_wait0);
      atomicAdd(a.stamps + 8 * a.ntasks_pairs + 3 * pd.slot + 1, n_wait);
      atomicAdd(a.stamps + 8 * a.ntasks_pairs + 3 * pd.slot + 2, (u64)nsb);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned prev = 0;
    if (lane == 0) prev = __hip_atomic_fetch_add((gu32*)(a.done + pd.slot), 1u, BITS_RLX);
    prev = __builtin_amdgcn_readfirstlane(prev);
    if (prev + 1u == (unsigned)pd.nbands) {  // the pair's last band: every band has released
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      BITS_PROG(0x40000000u);
      if (a.stamps && lane == 0) a.stamps[8 * pd.slot] = __builtin_amdgcn_s_memrealtime();
      int tlen;
      int2 tend;
      bool tout;
      // the walk is one wave's chain of dependent scalar instructions, and the fill
      // waves around it issue ~24 scalar instructions a step: it goes first
      // (NWK_COL_TRACE_PRIO=0 at build time: no raise, for A/B)
#if !defined(NWK_COL_TRACE_PRIO) || NWK_COL_TRACE_PRIO
      __builtin_amdgcn_s_setprio(3);
#endif
      if (pd.bits_w > 0) trace_col<false, true>(a, pd, obuf_all[wid], pf_all[wid], lane, 0, tlen, tend, tout);
      else trace_col<false, false>(a, pd, obuf_all[wid], pf_all[wid], lane, 0, tlen, tend, tout);
      if constexpr (FUSE) {
        // the first pieces of a streamed shard: rows, hash and record at once,
        // still at the walk's priority (rank 0's chain waits for these records)
        const bool early = a.early_hash > 0 && pd.prio >= a.early_hash;
        if (!early) __builtin_amdgcn_s_setprio(0);
        const bool ok_rows = !tout && fin_rows(a, pd, lane, tlen, tend);
        hq_push(a, pd, lane, ok_rows);
        if (early) hq_hash(a, lane, true);
      }
      __builtin_amdgcn_s_setprio(0);
      if (a.stamps && lane == 0) a.stamps[8 * pd.slot + 1] = __builtin_amdgcn_s_memrealtime();
      BITS_PROG(0x56000000u);
    } else if (pd.spec_every > 0 && band + 1 < pd.nbands) {  // segmented: this band's speculative segment
      int tlen;
      int2 tend;
      bool tout;
      __builtin_amdgcn_s_setprio(3);
      if (pd.bits_w > 0) trace_col<true, true>(a, pd, obuf_all[wid], pf_all[wid], lane, band, tlen, tend, tout);
      else trace_col<true, false>(a, pd, obuf_all[wid], pf_all[wid], lane, band, tlen, tend, tout);
      __builtin_amdgcn_s_setprio(0);
    }
  }
}

template <int NP, int SR>
hipError_t col_launch(const FillArgs& a, int grid, bool hi, hipStream_t s) {
#ifdef NWK_COL_NOFUSE
  if (a.fuse_fin) return hipErrorInvalidValue;
#else
  if (a.fuse_fin) hipLaunchKernelGGL((nw_align_col<NP, SR, true, NWK_COL_WPE>), dim3(grid), dim3(256), 0, s, a);
  else
#endif
  if (hi) hipLaunchKernelGGL((nw_align_col<NP, SR, false, NWK_COL_WPE_HI>), dim3(grid), dim3(256), 0, s, a);
  else hipLaunchKernelGGL((nw_align_col<NP, SR, false, NWK_COL_WPE>), dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int NP, int SR>
int col_occ(bool hi) {
  int n = 0;
  const void* k = hi ? reinterpret_cast<const void*>(&nw_align_col<NP, SR, false, NWK_COL_WPE_HI>)
                     : reinterpret_cast<const void*>(&nw_align_col<NP, SR, false, NWK_COL_WPE>);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 256, 0) != hipSuccess) return 1;
  return n > 0 ? n : 1;
}

}  // namespace

int bits_sr(int pxy, int pgap);

hipError_t launch_col(const FillArgs& a, int pxy, int pgap, int grid, bool hi, hipStream_t s) {
  const int sr = bits_sr(pxy, pgap);
#ifdef NWK_COL_ONE  // (development: one instantiation, fast builds)
  return pgap == 2 && sr == 1 ? col_launch<4, 1>(a, grid, hi, s) : hipErrorInvalidValue;
#endif
  if (pgap == 1) {
    switch (sr) {
      case -1: return col_launch<2, -1>(a, grid, hi, s);
      case 0: return col_launch<2, 0>(a, grid, hi, s);
      case 1: return col_launch<2, 1>(a, grid, hi, s);
      default: return col_launch<2, 2>(a, grid, hi, s);
    }
  }
  if (pgap == 2) {
    switch (sr) {
      case -1: return col_launch<4, -1>(a, grid, hi, s);
      case 0: return col_launch<4, 0>(a, grid, hi, s);
      case 1: return col_launch<4, 1>(a, grid, hi, s);
      case 2: return col_launch<4, 2>(a, grid, hi, s);
      case 3: return col_launch<4, 3>(a, grid, hi, s);
      default: return col_launch<4, 4>(a, grid, hi, s);
    }
  }
  return hipErrorInvalidValue;
}

int col_blocks_per_cu(int pgap, bool hi) { return pgap == 1 ? col_occ<2, 1>(hi) : col_occ<4, 1>(hi); }

}  // namespace nwk
