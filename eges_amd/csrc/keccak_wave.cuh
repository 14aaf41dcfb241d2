// Keccak-f[1600] with the state spread over the lanes of one wave (latency kernels).
//
// Same permutation as keccak.cuh (the reference's crypto/sha3 keccakf.go; sponge of sha3.go,
// rate 136, domain byte 0x01, hashes.go:16). The lane-serial form costs one wave ~4.5k dependent
// scalar instructions per address at the end of every latency-kernel signature; here the state
// is spread over the wave (lane x + 5y holds A[x, y], as 32-bit halves in the default form below),
// so a round is a few dozen VALU instructions and 11 dword gathers (ds_bpermute: the column
// parities, theta's neighbours, pi, chi's neighbours) in four dependent steps.
#pragma once
#include "keccak.cuh"

namespace eges {

// rho offsets by source lane x + 5y (keccak_f1600's rotl64 amounts)
__constant__ const uint32_t KECCAK_RHO[25] = {0,  1,  62, 28, 27, 36, 44, 6,  55, 20, 3,  10, 43,
                                              25, 39, 41, 45, 15, 21, 8,  18, 2,  61, 56, 14};

DEV uint64_t wave_gather64(uint64_t v, int addr) {  // v of lane addr / 4
  const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)(uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// The rounds are bound by ds_bpermute issue (a form with fewer dependent steps but more gathers
// was slower), so the state is held as 32-bit halves: lane x + 5y the low half of A[x, y], lane
// 32 + x + 5y the high half, and every gather moves one dword. Rotations need the other half of
// the same word: theta's rotl(C[x + 1], 1) gathers it beside C[x + 1], and rho is applied after
// pi from both halves of the source word (funnel shifts). 11 dword gathers per round instead
// of 18, in the same four dependent steps.
DEV uint32_t wave_gather32(uint32_t v, int addr) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)v);
}

// v: lane x + 5y (+ 32 for the high half) holds its half of A[x, y]; lanes 25..31, 57..63 anything
DEV void keccak_f1600_halves(uint32_t& v) {
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const int h = (int)(lane >> 5), l5 = (int)(lane & 31);
  const int li = l5 < 25 ? l5 : 0;
  const int x = li % 5, y = li / 5;
  const int base = 128 * h, obase = 128 * (1 - h);  // byte address of lane 0 of this / the other half
  const int c1 = base + 4 * (x + 5 * ((y + 1) % 5)), c2 = base + 4 * (x + 5 * ((y + 2) % 5));
  const int c3 = base + 4 * (x + 5 * ((y + 3) % 5)), c4 = base + 4 * (x + 5 * ((y + 4) % 5));
  const int xm1 = base + 4 * ((x + 4) % 5 + 5 * y), xp1 = base + 4 * ((x + 1) % 5 + 5 * y);
  const int xp1o = obase + 4 * ((x + 1) % 5 + 5 * y), xp2 = base + 4 * ((x + 2) % 5 + 5 * y);
  // pi: B[X, Y] = rotl(A'[x, y], rho[x, y]) with X = y, Y = 2x + 3y: lane X + 5Y reads lane
  // (X + 3Y) % 5 + 5X, both halves, and applies that lane's rho
  const int src = (x + 3 * y) % 5 + 5 * x;
  const int pis = base + 4 * src, piso = obase + 4 * src;
  const uint32_t r = KECCAK_RHO[src], sh = r & 31;
  const bool low_first = r < 32;  // rotl by r < 32: this half leads; by r >= 32: the other one
  const uint32_t rc_shift = 32 * (uint32_t)h;
#pragma unroll 1
  for (int round = 0; round < 24; ++round) {
    // theta: C[x] = xor over y of A[x, y]; A ^= C[x - 1] ^ rotl(C[x + 1], 1)
    const uint32_t c = v ^ wave_gather32(v, c1) ^ wave_gather32(v, c2) ^ wave_gather32(v, c3) ^ wave_gather32(v, c4);
    const uint32_t cm = wave_gather32(c, xm1), cp = wave_gather32(c, xp1), cpo = wave_gather32(c, xp1o);
    v ^= cm ^ ((cp << 1) | (cpo >> 31));
    // pi, then the source word's rho as a funnel shift of its two halves
    const uint32_t t = wave_gather32(v, pis), o = wave_gather32(v, piso);
    const uint32_t hi = low_first ? t : o, lo = low_first ? o : t;
    const uint32_t b = sh == 0 ? hi : __builtin_amdgcn_alignbit(hi, lo, 32 - sh);
    // chi, iota
    v = b ^ (~wave_gather32(b, xp1) & wave_gather32(b, xp2));
    if (l5 == 0) v ^= (uint32_t)(KECCAK_RC[round] >> rc_shift);
  }
}

// a: this lane's state word A[x + 5y] for lanes 0..24 (other lanes: anything); on return
// lanes 0..24 hold the permuted state
DEV void keccak_f1600_wave(uint64_t& a) {
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const uint32_t hi_in = wave_gather32((uint32_t)(a >> 32), (int)(4 * (lane & 31)));
  uint32_t v = lane < 32 ? (uint32_t)a : hi_in;
  keccak_f1600_halves(v);
  const uint32_t hi_out = wave_gather32(v, (int)(4 * ((lane & 31) + 32)));
  a = ((uint64_t)hi_out << 32) | v;
}

// Keccak-256(X || Y)[12:32] as 5 little-endian words, X and Y canonical and wave-uniform
// (core.cuh pub_address, computed across the lanes of the wave).
DEV void pub_address_wave(uint32_t out[5], const uint32_t X[8], const uint32_t Y[8]) {
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  uint64_t a = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    a = lane == (uint32_t)k ? be_word(X, k) : a;
    a = lane == (uint32_t)(4 + k) ? be_word(Y, k) : a;
  }
  a ^= lane == 8 ? 0x01ull : 0ull;           // pad: byte 64 ^= 0x01
  a ^= lane == 16 ? (0x80ull << 56) : 0ull;  //      byte 135 ^= 0x80
  keccak_f1600_wave(a);
  const uint32_t lo = (uint32_t)a, hi = (uint32_t)(a >> 32);
  out[0] = (uint32_t)__builtin_amdgcn_readlane((int)hi, 1);
  out[1] = (uint32_t)__builtin_amdgcn_readlane((int)lo, 2);
  out[2] = (uint32_t)__builtin_amdgcn_readlane((int)hi, 2);
  out[3] = (uint32_t)__builtin_amdgcn_readlane((int)lo, 3);
  out[4] = (uint32_t)__builtin_amdgcn_readlane((int)hi, 3);
}

}  // namespace eges
