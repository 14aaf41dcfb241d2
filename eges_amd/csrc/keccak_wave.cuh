// Keccak-f[1600] with the state spread over the lanes of one wave (latency kernels).
//
// Same permutation as keccak.cuh (the reference's crypto/sha3 keccakf.go; sponge of sha3.go,
// rate 136, domain byte 0x01, hashes.go:16). The lane-serial form costs one wave ~4.5k dependent
// scalar instructions per address at the end of every latency-kernel signature; here lane
// x + 5y holds A[x, y] (lanes 25..63 idle), so a round is ~25 VALU instructions and nine
// cross-lane gathers (ds_bpermute: the column parities, theta's neighbours, pi, chi's
// neighbours) in four dependent steps.
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

// a: this lane's state word A[x + 5y] for lanes 0..24 (other lanes: anything)
DEV void keccak_f1600_wave(uint64_t& a) {
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const int li = lane < 25 ? (int)lane : 0;
  const int x = li % 5, y = li / 5;
  // byte addresses of the lanes each step reads
  const int c1 = 4 * (x + 5 * ((y + 1) % 5)), c2 = 4 * (x + 5 * ((y + 2) % 5));
  const int c3 = 4 * (x + 5 * ((y + 3) % 5)), c4 = 4 * (x + 5 * ((y + 4) % 5));
  const int xm1 = 4 * ((x + 4) % 5 + 5 * y), xp1 = 4 * ((x + 1) % 5 + 5 * y), xp2 = 4 * ((x + 2) % 5 + 5 * y);
  // pi: B[X, Y] = A'[x, y] with X = y, Y = 2x + 3y, i.e. lane X + 5Y reads lane (X + 3Y) % 5 + 5X
  const int pis = 4 * ((x + 3 * y) % 5 + 5 * x);
  const uint32_t rho = KECCAK_RHO[li];
#pragma unroll 1
  for (int round = 0; round < 24; ++round) {
    // theta: C[x] = xor over y of A[x, y]; A ^= C[x - 1] ^ rotl(C[x + 1], 1)
    const uint64_t c = a ^ wave_gather64(a, c1) ^ wave_gather64(a, c2) ^ wave_gather64(a, c3) ^ wave_gather64(a, c4);
    const uint64_t cp = wave_gather64(c, xp1);
    a ^= wave_gather64(c, xm1) ^ rotl64(cp, 1);
    // rho (this lane's offset; 0 on lane 0), then pi
    a = (a << rho) | (a >> ((64 - rho) & 63));
    const uint64_t b = wave_gather64(a, pis);
    // chi, iota
    a = b ^ (~wave_gather64(b, xp1) & wave_gather64(b, xp2));
    if (lane == 0) a ^= KECCAK_RC[round];
  }
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
