// Band geometry of nw_profile (the MSA's profile-profile fill, nwk_kernels.hip)
// and of its walk, trace_pair_affine<true, kProfRows>; shared with nwk_msa's
// host side (nwk_runtime.cpp), which sizes the bands and their code storage.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef NWK_PROF_ROWS
#define NWK_PROF_ROWS 4
#endif
// DP rows per lane: a band is 64 lanes x kProfRows rows. 4 (round 6; was the
// pairwise kernels' kRows = 8): a level's merge runs twice the waves, each step
// half the rows.
constexpr int kProfRows = NWK_PROF_ROWS;
constexpr int kProfBandRows = 64 * kProfRows;
static_assert(kProfRows == 4 || kProfRows == 8, "nw_profile: 4 or 8 rows per lane");
// one band's 4-bit codes: a dword holds 8 steps of one row of one lane, in
// column units of kProfRows x 64 dwords; sblocks super-blocks of 64 steps
__host__ __device__ inline int64_t prof_band_dwords(int sblocks) { return (int64_t)sblocks * 8 * kProfRows * 64; }
