// nwk_gotoh_planes.h -- the bit-sliced Gotoh step of nw_align_gotoh
// (nwk_gotoh.hip; also compiled on the host by tools/probe/gotoh_sim.cpp, whose
// test pins the algebra cell by cell).  One call evaluates 32 cells, one per
// bit, of the affine recurrence (oracle/nw_oracle.c nwo_pair_affine):
//   E = min(E_left + ge, H_left + go + ge),  F = min(F_up + ge, H_up + go + ge),
//   H = min(H_diag + (match ? 0 : pxy), E, F).
//
// G-space (G = H - (i + j) ge, E' and F' likewise) removes ge from the gaps:
//   E' = min(E'_left, G_left + go),  F' = min(F'_up, G_up + go),
//   G  = min(G_diag + s - 2 ge, E', F').
// Relative to G_diag, with the differences
//   L = v(i, j-1) = G(i-1, j-1) - G(i, j-1)   (vertical, from the left cell)
//   U = h(i-1, j) = G(i-1, j-1) - G(i-1, j)   (horizontal, from the upper cell)
//   eL = E'(i, j-1) - G(i, j-1) >= 0,  fU = F'(i-1, j) - G(i-1, j) >= 0
// the cell is X = G_diag - G = max(S, a, b) with S = 2 ge - s,
//   a = L - min(eL, go) (= G_diag - E'),  b = U - min(fU, go) (= G_diag - F'),
// and its outputs are
//   v = X - U,  h = X - L,  e = X - a = h + min(eL, go),  f = v + min(fU, go).
// Only min(e, go) and min(f, go) are ever read, so e and f saturate at go.
//
// Thermometer planes: a difference x in [VLO, VHI] (VLO = -go, VHI = go + 2 ge)
// is held as P[p] = [x >= VLO + 1 + p]; a saturated gap offset as Q[q - 1] =
// [x >= q], q = 1 .. go.  Every output plane is an OR of (plane AND NOT plane)
// terms, so max is OR and differences are the convolutions below.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GB_HD __host__ __device__ __forceinline__
#else
#define GB_HD inline
#endif

namespace gotoh_bits {

template <int GO, int GE, int PXY>
struct Cfg {
  static constexpr int VLO = -GO, VHI = GO + 2 * GE;  // range of v and h
  static constexpr int NV = VHI - VLO;                // planes of v / h
  static constexpr int NQ = GO;                       // planes of min(e, go) / min(f, go)
  static constexpr int SM = 2 * GE, SX = 2 * GE - PXY;  // S on a match / mismatch
  static constexpr int XLO = SX, XHI = VHI;           // X >= S >= SX; X <= max(SM, VHI)
  static constexpr int NX = XHI - XLO;                // planes of X: [X >= XLO + 1 + p]
  static_assert(PXY >= 0 && GE >= 1 && GO >= 0, "domain of the probe");
  static_assert(SM <= VHI, "X's top must be VHI");
};

// Operand kinds, known at compile time: Z all zeros, O all ones, P a plane.
enum { kZ = 0, kO = 1, kP = 2 };
template <class C, int c>
constexpr int kind_v() { return c <= C::VLO ? kO : (c > C::VHI ? kZ : kP); }
template <class C, int q>
constexpr int kind_q() { return q <= 0 ? kO : (q > C::NQ ? kZ : kP); }
template <class C, int c>
constexpr int kind_x() { return c <= C::XLO ? kO : (c > C::XHI ? kZ : kP); }

// [x >= c] of a difference held as NV planes
template <class C, int c>
GB_HD uint32_t ge_v(const uint32_t (&P)[C::NV]) {
  if constexpr (kind_v<C, c>() == kO) return ~0u;
  else if constexpr (kind_v<C, c>() == kZ) return 0u;
  else return P[c - C::VLO - 1];
}
// [x >= q] of a gap offset saturated at go
template <class C, int q>
GB_HD uint32_t ge_q(const uint32_t (&Q)[C::NQ > 0 ? C::NQ : 1]) {
  if constexpr (kind_q<C, q>() == kO) return ~0u;
  else if constexpr (kind_q<C, q>() == kZ) return 0u;
  else return Q[q - 1];
}
template <class C, int c>
GB_HD uint32_t ge_x(const uint32_t (&X)[C::NX]) {
  if constexpr (kind_x<C, c>() == kO) return ~0u;
  else if constexpr (kind_x<C, c>() == kZ) return 0u;
  else return X[c - C::XLO - 1];
}

// acc | (a & b') with b' = NB ? ~b : b, one v_bitop3_b32 when both operands
// are planes and acc holds earlier terms (HAS); constant operands fold away.
#if defined(__HIP_DEVICE_COMPILE__)
#define GB_OR_AND(acc, a, b) __builtin_amdgcn_bitop3_b32((acc), (a), (b), 0xF0u | (0xCCu & 0xAAu))
#define GB_OR_ANDN(acc, a, b) __builtin_amdgcn_bitop3_b32((acc), (a), (b), 0xF0u | (0xCCu & ~0xAAu & 0xFFu))
#define GB_OR_NOT(acc, b) __builtin_amdgcn_bitop3_b32((acc), (b), (b), 0xF0u | (~0xCCu & 0xFFu))
#define GB_ANDN(a, b) __builtin_amdgcn_bitop3_b32((a), (b), (b), 0xF0u & ~0xCCu & 0xFFu)
#else
#define GB_OR_AND(acc, a, b) ((acc) | ((a) & (b)))
#define GB_OR_ANDN(acc, a, b) ((acc) | ((a) & ~(b)))
#define GB_OR_NOT(acc, b) ((acc) | ~(b))
#define GB_ANDN(a, b) ((a) & ~(b))
#endif
template <int KA, int KB, bool NB>
constexpr bool term_nonzero() {
  constexpr int kb = NB ? (KB == kZ ? kO : (KB == kO ? kZ : kP)) : KB;
  return KA != kZ && kb != kZ;
}
template <int KA, int KB, bool NB, bool HAS>
GB_HD uint32_t acc_term(uint32_t acc, uint32_t a, uint32_t b) {
  constexpr int kb = NB ? (KB == kZ ? kO : (KB == kO ? kZ : kP)) : KB;  // kind of b'
  if constexpr (KA == kZ || kb == kZ) {
    return acc;
  } else if constexpr (KA == kO && kb == kO) {
    return ~0u;
  } else if constexpr (KA == kO) {  // the term is b'
    const uint32_t t = NB ? ~b : b;
    if constexpr (HAS) return NB ? GB_OR_NOT(acc, b) : (acc | b);
    else return t;
  } else if constexpr (kb == kO) {  // the term is a
    if constexpr (HAS) return acc | a;
    else return a;
  } else {
    if constexpr (HAS) return NB ? GB_OR_ANDN(acc, a, b) : GB_OR_AND(acc, a, b);
    else return NB ? GB_ANDN(a, b) : (a & b);
  }
}

// [Lv - min(e, go) >= c] = OR_{q=0..go} ([e <= q] & [Lv >= c + q]), accumulated
// onto acc: term q is Lv_{c+q} & ~E_{q+1}.  Taken from q = go down: term go is
// the plane Lv_{c+go} alone, which then starts the accumulator for free.
template <class C, int c, bool HAS, int q = C::NQ>
GB_HD uint32_t sub_gap(uint32_t acc, const uint32_t (&Lv)[C::NV], const uint32_t (&E)[C::NQ > 0 ? C::NQ : 1]) {
  constexpr int KA = kind_v<C, c + q>(), KB = kind_q<C, q + 1>();
  const uint32_t r = acc_term<KA, KB, true, HAS>(acc, ge_v<C, c + q>(Lv), ge_q<C, q + 1>(E));
  constexpr bool has = HAS || term_nonzero<KA, KB, true>();
  if constexpr (q <= 0) return r;
  else return sub_gap<C, c, has, q - 1>(r, Lv, E);
}
template <class C, int c, int q = 0>
constexpr bool sub_gap_any() {
  if constexpr (q > C::NQ) return false;
  else return term_nonzero<kind_v<C, c + q>(), kind_q<C, q + 1>(), true>() || sub_gap_any<C, c, q + 1>();
}

// [X - Y >= c] = OR_{d = XLO..XHI} ([X >= d] & ~[Y >= d - c + 1]).  Taken
// from d = XHI down: term XLO is ~Y alone ([X >= XLO] holds), which then joins
// the accumulator in the same instruction (acc | ~Y) instead of a v_not first.
template <class C, int c, bool HAS = false, int d = C::XHI>
GB_HD uint32_t diff_xv(uint32_t acc, const uint32_t (&X)[C::NX], const uint32_t (&Y)[C::NV]) {
  constexpr int KA = kind_x<C, d>(), KB = kind_v<C, d - c + 1>();
  const uint32_t r = acc_term<KA, KB, true, HAS>(acc, ge_x<C, d>(X), ge_v<C, d - c + 1>(Y));
  constexpr bool has = HAS || term_nonzero<KA, KB, true>();
  if constexpr (d <= C::XLO) return has ? r : 0u;
  else return diff_xv<C, c, has, d - 1>(r, X, Y);
}

// [Y + min(e, go) >= q] = OR_{r=0..go} ([e >= r] & [Y >= q - r])
template <class C, int q, bool HAS = false, int r = 0>
GB_HD uint32_t add_gap(uint32_t acc, const uint32_t (&Y)[C::NV], const uint32_t (&E)[C::NQ > 0 ? C::NQ : 1]) {
  constexpr int KA = kind_v<C, q - r>(), KB = kind_q<C, r>();
  const uint32_t t = acc_term<KA, KB, false, HAS>(acc, ge_v<C, q - r>(Y), ge_q<C, r>(E));
  constexpr bool has = HAS || term_nonzero<KA, KB, false>();
  if constexpr (r >= C::NQ) return has ? t : 0u;
  else return add_gap<C, q, has, r + 1>(t, Y, E);
}

template <class C, int p = 0>
GB_HD void x_planes(uint32_t match, const uint32_t (&L)[C::NV], const uint32_t (&eL)[C::NQ > 0 ? C::NQ : 1],
                    const uint32_t (&U)[C::NV], const uint32_t (&fU)[C::NQ > 0 ? C::NQ : 1], uint32_t (&X)[C::NX]) {
  if constexpr (p < C::NX) {
    constexpr int c = C::XLO + 1 + p;
    // [S >= c] first (ones, the match plane or nothing), then a's and b's terms
    constexpr int KS = c <= C::SX ? kO : (c <= C::SM ? kP : kZ);
    const uint32_t s0 = KS == kO ? ~0u : (KS == kP ? match : 0u);
    constexpr bool hs = KS != kZ;
    const uint32_t ra = sub_gap<C, c, hs>(s0, L, eL);
    constexpr bool ha = hs || sub_gap_any<C, c>();
    const uint32_t rb = sub_gap<C, c, ha>(ra, U, fU);
    X[p] = (ha || sub_gap_any<C, c>()) ? rb : 0u;
    x_planes<C, p + 1>(match, L, eL, U, fU, X);
  }
}
template <class C, int p = 0>
GB_HD void v_planes(const uint32_t (&X)[C::NX], const uint32_t (&Y)[C::NV], uint32_t (&out)[C::NV]) {
  if constexpr (p < C::NV) {
    out[p] = diff_xv<C, C::VLO + 1 + p>(0u, X, Y);
    v_planes<C, p + 1>(X, Y, out);
  }
}
template <class C, int q = 1>
GB_HD void q_planes(const uint32_t (&Y)[C::NV], const uint32_t (&E)[C::NQ > 0 ? C::NQ : 1],
                    uint32_t (&out)[C::NQ > 0 ? C::NQ : 1]) {
  if constexpr (q <= C::NQ) {
    out[q - 1] = add_gap<C, q>(0u, Y, E);
    q_planes<C, q + 1>(Y, E, out);
  }
}

// One step for 32 cells.  In: L, eL (left cells), U, fU (upper cells), match.
// Out: v, e (to the right), h, f (down), and the traceback bits the oracle's
// walk reads (nwo_pair_affine: D > F > E on ties, a gap opens on a tie):
//   D    = [G == G_diag + s - 2 ge]          (X == S)
//   Fsrc = [G == F']                         (f == 0)
//   Eext = [E' came from E'_left]            (eL < go)
//   Fext = [F' came from F'_up]              (fU < go)
template <class C>
GB_HD void step(uint32_t match, const uint32_t (&L)[C::NV], const uint32_t (&eL)[C::NQ > 0 ? C::NQ : 1],
                const uint32_t (&U)[C::NV], const uint32_t (&fU)[C::NQ > 0 ? C::NQ : 1], uint32_t (&v)[C::NV],
                uint32_t (&e)[C::NQ > 0 ? C::NQ : 1], uint32_t (&h)[C::NV], uint32_t (&f)[C::NQ > 0 ? C::NQ : 1],
                uint32_t& D, uint32_t& Fsrc, uint32_t& Eext, uint32_t& Fext) {
  uint32_t X[C::NX];
  x_planes<C>(match, L, eL, U, fU, X);
  v_planes<C>(X, U, v);
  v_planes<C>(X, L, h);
  q_planes<C>(h, eL, e);
  q_planes<C>(v, fU, f);
  D = (match & ~ge_x<C, C::SM + 1>(X)) | (~match & ~ge_x<C, C::SX + 1>(X));
  Fsrc = ~add_gap<C, 1>(0u, v, fU);  // ~[f >= 1] (f's plane 0; go = 0 keeps no f planes)
  Eext = ~ge_q<C, C::NQ>(eL);
  Fext = ~ge_q<C, C::NQ>(fU);
  if constexpr (C::NQ == 0) {  // go = 0: every gap cell may open (ties open)
    e[0] = f[0] = 0u;
    Eext = Fext = 0u;
  }
}

// planes of a constant difference / saturated gap offset
template <class C>
GB_HD void const_v(int x, uint32_t (&P)[C::NV]) {
  for (int p = 0; p < C::NV; ++p) P[p] = x >= C::VLO + 1 + p ? ~0u : 0u;
}
template <class C>
GB_HD void const_q(int x, uint32_t (&Q)[C::NQ > 0 ? C::NQ : 1]) {
  for (int q = 1; q <= C::NQ; ++q) Q[q - 1] = x >= q ? ~0u : 0u;
  if constexpr (C::NQ == 0) Q[0] = 0u;
}

}  // namespace gotoh_bits
