// Keccak-f[1600] and single-block Keccak-256 for gfx950.
//
// Same function as the reference's crypto/sha3 (keccakf.go / keccakf_amd64.s permutation;
// sponge of sha3.go with rate 136 and domain byte 0x01, hashes.go:16). 64-bit lanes are
// split by the compiler into 32-bit halves; rotations lower to v_alignbit_b32 pairs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef DEV
#define DEV __device__ __forceinline__
#endif

namespace eges {

__constant__ const uint64_t KECCAK_RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};

DEV uint64_t rotl64(uint64_t x, int n) { return (x << n) | (x >> (64 - n)); }

// A[x + 5y]
DEV void keccak_f1600(uint64_t A[25]) {
#pragma unroll 1
  for (int round = 0; round < 24; ++round) {
    uint64_t C0 = A[0] ^ A[5] ^ A[10] ^ A[15] ^ A[20];
    uint64_t C1 = A[1] ^ A[6] ^ A[11] ^ A[16] ^ A[21];
    uint64_t C2 = A[2] ^ A[7] ^ A[12] ^ A[17] ^ A[22];
    uint64_t C3 = A[3] ^ A[8] ^ A[13] ^ A[18] ^ A[23];
    uint64_t C4 = A[4] ^ A[9] ^ A[14] ^ A[19] ^ A[24];
    uint64_t D0 = C4 ^ rotl64(C1, 1);
    uint64_t D1 = C0 ^ rotl64(C2, 1);
    uint64_t D2 = C1 ^ rotl64(C3, 1);
    uint64_t D3 = C2 ^ rotl64(C4, 1);
    uint64_t D4 = C3 ^ rotl64(C0, 1);
    // theta + rho + pi: B[y, 2x+3y] = rot(A[x,y] ^ D[x], r[x,y])
    uint64_t B00 = A[0] ^ D0;
    uint64_t B10 = rotl64(A[6] ^ D1, 44);
    uint64_t B20 = rotl64(A[12] ^ D2, 43);
    uint64_t B30 = rotl64(A[18] ^ D3, 21);
    uint64_t B40 = rotl64(A[24] ^ D4, 14);
    uint64_t B01 = rotl64(A[3] ^ D3, 28);
    uint64_t B11 = rotl64(A[9] ^ D4, 20);
    uint64_t B21 = rotl64(A[10] ^ D0, 3);
    uint64_t B31 = rotl64(A[16] ^ D1, 45);
    uint64_t B41 = rotl64(A[22] ^ D2, 61);
    uint64_t B02 = rotl64(A[1] ^ D1, 1);
    uint64_t B12 = rotl64(A[7] ^ D2, 6);
    uint64_t B22 = rotl64(A[13] ^ D3, 25);
    uint64_t B32 = rotl64(A[19] ^ D4, 8);
    uint64_t B42 = rotl64(A[20] ^ D0, 18);
    uint64_t B03 = rotl64(A[4] ^ D4, 27);
    uint64_t B13 = rotl64(A[5] ^ D0, 36);
    uint64_t B23 = rotl64(A[11] ^ D1, 10);
    uint64_t B33 = rotl64(A[17] ^ D2, 15);
    uint64_t B43 = rotl64(A[23] ^ D3, 56);
    uint64_t B04 = rotl64(A[2] ^ D2, 62);
    uint64_t B14 = rotl64(A[8] ^ D3, 55);
    uint64_t B24 = rotl64(A[14] ^ D4, 39);
    uint64_t B34 = rotl64(A[15] ^ D0, 41);
    uint64_t B44 = rotl64(A[21] ^ D1, 2);
    // chi: A[x,y] = B[x,y] ^ (~B[x+1,y] & B[x+2,y]); row y holds B0y..B4y
    A[0] = B00 ^ (~B10 & B20);
    A[1] = B10 ^ (~B20 & B30);
    A[2] = B20 ^ (~B30 & B40);
    A[3] = B30 ^ (~B40 & B00);
    A[4] = B40 ^ (~B00 & B10);
    A[5] = B01 ^ (~B11 & B21);
    A[6] = B11 ^ (~B21 & B31);
    A[7] = B21 ^ (~B31 & B41);
    A[8] = B31 ^ (~B41 & B01);
    A[9] = B41 ^ (~B01 & B11);
    A[10] = B02 ^ (~B12 & B22);
    A[11] = B12 ^ (~B22 & B32);
    A[12] = B22 ^ (~B32 & B42);
    A[13] = B32 ^ (~B42 & B02);
    A[14] = B42 ^ (~B02 & B12);
    A[15] = B03 ^ (~B13 & B23);
    A[16] = B13 ^ (~B23 & B33);
    A[17] = B23 ^ (~B33 & B43);
    A[18] = B33 ^ (~B43 & B03);
    A[19] = B43 ^ (~B03 & B13);
    A[20] = B04 ^ (~B14 & B24);
    A[21] = B14 ^ (~B24 & B34);
    A[22] = B24 ^ (~B34 & B44);
    A[23] = B34 ^ (~B44 & B04);
    A[24] = B44 ^ (~B04 & B14);
    A[0] ^= KECCAK_RC[round];
  }
}

// Keccak-256 of a message of at most 135 bytes given as little-endian 64-bit words
// (NBYTES bytes valid, the rest of the 17 words must be zero); writes the 4 digest lanes.
template <int NBYTES>
DEV void keccak256_1block(const uint64_t* words, uint64_t out[4]) {
  static_assert(NBYTES < 136, "single block only");
  uint64_t A[25];
#pragma unroll
  for (int i = 0; i < 25; ++i) A[i] = i < 17 ? words[i] : 0;
  // pad: byte nbytes ^= 0x01, byte 135 ^= 0x80
  A[NBYTES >> 3] ^= 0x01ull << (8 * (NBYTES & 7));
  A[16] ^= 0x80ull << 56;
  keccak_f1600(A);
#pragma unroll
  for (int i = 0; i < 4; ++i) out[i] = A[i];
}

}  // namespace eges
