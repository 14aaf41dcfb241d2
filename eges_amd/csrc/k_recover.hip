#include <type_traits>

#include "core.cuh"
#include "modinv_row.cuh"

#ifndef EGES_LS_BATCHINV
#define EGES_LS_BATCHINV 1  // phases B / D across the wave (sc_inv_wave / fe_inv_wave_z); 0: per thread
#endif

namespace eges {

// ------------------------------------------------------------------ host-buffer form
// Block 0 of a host-buffer launch (RecoverParams::ls_host): one wave copies the host's piece count
// into the device word the signature waves poll, until the last piece (or 4 s). A single poller
// of the bus word: every wave polling it over PCIe would flood the link.
DEV void ls_mirror(const RecoverParams& prm) {
  if (threadIdx.x >= 64) return;
  uint32_t* h = const_cast<uint32_t*>(prm.ls_host);
  constexpr uint64_t BOUND = 400000000ull;  // s_memrealtime ticks (100 MHz): 4 s
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t last = prm.ls_seq;
#pragma unroll 1
  for (;;) {
    const uint32_t v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    if (v != last) {
      if (threadIdx.x == 0) __hip_atomic_store(prm.ls_arrived, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = v;
    }
    if ((int32_t)(v - prm.ls_final) >= 0) return;
    if (__builtin_amdgcn_s_memrealtime() - t0 > BOUND) {
      if (threadIdx.x == 0) {
        __hip_atomic_store(prm.ls_fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(prm.ls_arrived, prm.ls_final, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // release the waves
      }
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}
// Wait until piece `piece` has been written (RecoverParams::ls_arrived, mirrored by block 0). The
// piece is wave-uniform; the inputs are read only after it (no line of them was read before in
// this launch, whose start invalidated the caches).
DEV void ls_wait(const RecoverParams& prm, uint32_t piece) {
  const uint32_t want = prm.ls_seq + piece + 1u;
  constexpr uint64_t BOUND = 500000000ull;  // s_memrealtime ticks (100 MHz): 5 s (the mirror gives up at 4)
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
  while ((int32_t)(__builtin_amdgcn_readfirstlane(
                       __hip_atomic_load(prm.ls_arrived, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) - want) < 0) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > BOUND) {
      if ((threadIdx.x & 63) == 0) __hip_atomic_store(prm.ls_fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}
// prep_ecrecover_kernel's parse (k_prep.hip) of item idx from the bytes, into its record rows
DEV void ls_parse(const RecoverParams& prm, uint32_t idx, uint32_t rl[8], uint32_t sl[8], uint32_t& meta) {
  const uint32_t np = prm.n_pad;
  uint32_t* rec = const_cast<uint32_t*>(prm.rec);
  const uint8_t* sg = prm.ls_sig + (size_t)idx * 65;
  uint32_t zl[8];
  limbs_from_be32(zl, prm.ls_msg + (size_t)idx * 32);
  limbs_from_be32(rl, sg);
  limbs_from_be32(sl, sg + 32);
  const uint32_t v = sg[64];
  meta = v >= 4 ? (ST_INVALID_RECOVERY_ID << 8) : v;  // checkSignature (secp256.go:171-179)
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    rec[(size_t)k * np + idx] = zl[k];
    rec[(size_t)(8 + k) * np + idx] = rl[k];
    rec[(size_t)(16 + k) * np + idx] = sl[k];
  }
  rec[(size_t)24 * np + idx] = meta;
}

// ------------------------------------------------------------------ recover kernel
// Lane-serial layout: the grid has GT = gridDim.x * WG threads and thread g owns the
// signatures idx = k * GT + g, k < K_g (K_g <= MAX_SLOTS). Each thread runs Montgomery's
// batch-inversion trick over its own K_g signatures, so the two exponentiations (r^-1 mod n and
// the final Z^-1 mod p) cost 1/K_g each per signature and run on all 64 lanes of every wave —
// no workgroup barrier, no idle waves. Per-signature state between the phases lives in the
// slot rows that follow the record rows (launch.h).
//
// Phase marks (diagnostic build only): 0 parse + sqrt, 1 r^-1 + u1/u2, 2 GLV + digits,
// 3 R table, 4 Strauss loop, 5 Z^-1, 6 affine + Keccak + stores.
//
template <class ST>
DEV void recover_body(const RecoverParams& prm, uint64_t* stamps) {
  __shared__ CoreLds L;
  ST st_;
  ST* st = &st_;
  uint4* const slot = recover_slots(prm.rec, prm.n_pad);
  const uint32_t np = prm.n_pad;
  const uint32_t bias = prm.ls_host ? 1u : 0u;  // host-buffer form: block 0 is the mirror
  const uint32_t GT = (gridDim.x - bias) * WG;
  const uint32_t g = (blockIdx.x - bias) * WG + threadIdx.x;
  const uint32_t K = g < prm.n ? (prm.n - g + GT - 1) / GT : 0;  // my signatures
  uint32_t okm = 0;
  const uint32_t units = 5u * K;
  // --- phase A: parse, lift R, prefix products of r
  sc pre = sc_one();
#pragma unroll 1
  for (uint32_t k = 0; k < K; ++k) {
    balance_prio(k, units);
    const uint32_t idx = k * GT + g;
    uint32_t rl[8], meta;
    bool ok, ovr, ovs;
    sc R;
    {
      uint32_t sl[8];
      if (prm.ls_msg) {  // host-buffer form: this slot's piece has arrived, then the parse
        ls_wait(prm, (g / prm.ls_group) * prm.ls_kmax + k);
        ls_parse(prm, idx, rl, sl, meta);
      } else {
        rec_get(prm, 8, idx, rl);
        rec_get(prm, 16, idx, sl);
        meta = prm.rec[(size_t)24 * np + idx];
      }
      ok = ((meta >> 8) & 0xffu) == ST_OK;
      // parse_compact: r, s >= n => failure (recovery/main_impl.h:38-58)
      R = sc_from_limbs(rl, ovr);
      const sc S = sc_from_limbs(sl, ovs);
      ok = ok && !ovr && !ovs && !sc_is_zero(R) && !sc_is_zero(S);
    }
    const uint32_t recid = meta & 3u;
    // x = r (+ n)  (main_impl.h:101-109)
    uint32_t xr[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) xr[i] = R.v[i];
    if (recid & 2u) {
      ok = ok && !u256_ge(R.v, P_MINUS_N);
      uint64_t c = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        c += (uint64_t)xr[i] + SC_N[i];
        xr[i] = (uint32_t)c;
        c >>= 32;
      }
    }
    ge Rp;
    ok = ge_set_xo(Rp, fe_from_u256(xr), (recid & 1u) != 0) && ok;
    // failed signatures carry the generator and r = 1 so every later step stays well-defined
    const ge G = gen_point();
    Rp.x = fe_select(ok, Rp.x, G.x);
    Rp.y = fe_select(ok, Rp.y, G.y);
    pre = sc_mul(pre, sc_select(ok, R, sc_one()));
    slot_put_pt(slot, np, 0, idx, Rp);
    slot_put_sc(slot, np, 5, idx, pre);
    okm |= (ok ? 1u : 0u) << k;
  }
  st->mark(0);
  // --- phase B: one scalar inversion per thread, or (EGES_LS_BATCHINV) one per wave: the 64
  // threads' products batched again across the lanes, inverted once by the row-form safegcd
  sc rinv_acc = EGES_LS_BATCHINV ? sc_inv_wave(pre) : sc_inv(pre);
  st->mark(1);
  // --- phase C: k = K-1 .. 0: r^-1, u1 = -z/r, u2 = s/r, Q = u2 R + u1 G, prefix products of Z
  fe zpre = fe_one();
#pragma unroll 1
  for (int k = (int)K - 1; k >= 0; --k) {
    balance_prio(K + 4u * (K - 1u - (uint32_t)k), units);
    const uint32_t idx = (uint32_t)k * GT + g;
    bool ok = (okm >> k) & 1u;
    sc rinv, u1, u2;
    {
      uint32_t l[8];
      bool ov;
      rec_get(prm, 8, idx, l);
      const sc R = sc_select(ok, sc_from_limbs(l, ov), sc_one());
      rinv = k > 0 ? sc_mul(rinv_acc, slot_get_sc(slot, np, 5, idx - GT)) : rinv_acc;
      rinv_acc = sc_mul(rinv_acc, R);
      rec_get(prm, 0, idx, l);
      const sc Z = sc_from_limbs(l, ov);  // msg mod n (main_impl.h:183)
      rec_get(prm, 16, idx, l);
      const sc S = sc_from_limbs(l, ov);
      u1 = sc_neg(sc_mul(rinv, Z));
      u2 = sc_select(ok, sc_mul(rinv, S), sc_one());
    }
    st->mark(1);
    const ge Rp = slot_get_pt(slot, np, 0, idx);
    park_put<8>(prm.ws, 0, rinv_acc.v);
    park_put<FE_LIMBS>(prm.ws, 8, zpre.v);
    gej Q;
    bool qinf;
    ecmult_core(Q, qinf, Rp, u2, u1, prm.gtab, prm.ws, L, st, diag_of(prm));
    park_get<8>(prm.ws, 0, rinv_acc.v);
    park_get<FE_LIMBS>(prm.ws, 8, zpre.v);
    ok = ok && !qinf;  // main_impl.h:120
    okm = (okm & ~(1u << k)) | ((ok ? 1u : 0u) << k);
    Q.z = fe_select(ok, Q.z, fe_one());
    zpre = fe_mul(zpre, Q.z);
    ge xy;
    xy.x = Q.x;
    xy.y = Q.y;
    slot_put_pt(slot, np, 0, idx, xy);
    ge zz;
    zz.x = Q.z;
    zz.y = zpre;
    slot_put_pt(slot, np, 7, idx, zz);
  }
  // --- phase D: one field inversion per thread (or per wave, as phase B)
  fe zinv_acc = EGES_LS_BATCHINV ? fe_inv_wave_z(zpre) : fe_inv(zpre);
  st->mark(5);
  // --- phase E: k = 0 .. K-1 (reverse of phase C's product order): affine, address, stores
#pragma unroll 1
  for (uint32_t k = 0; k < K; ++k) {
    const uint32_t idx = k * GT + g;
    const bool ok = (okm >> k) & 1u;
    const ge zz = slot_get_pt(slot, np, 7, idx);
    const fe zi = k + 1 < K ? fe_mul(zinv_acc, slot_get_pt(slot, np, 7, idx + GT).y) : zinv_acc;
    zinv_acc = fe_mul(zinv_acc, zz.x);
    const ge xy = slot_get_pt(slot, np, 0, idx);
    const fe zi2 = fe_sqr(zi);
    uint32_t X[8], Y[8];
    fe_to_u256(X, fe_normalize(fe_mul(xy.x, zi2)));
    fe_to_u256(Y, fe_normalize(fe_mul(xy.y, fe_mul(zi2, zi))));
    const uint32_t pre_st = (prm.rec[(size_t)24 * np + idx] >> 8) & 0xffu;
    prm.status[idx] = (uint8_t)(pre_st != ST_OK ? pre_st : (ok ? ST_OK : ST_RECOVER_FAILED));
    if (prm.addr) {
      uint32_t a[5];
      pub_address(a, X, Y);
      uint32_t* dst = reinterpret_cast<uint32_t*>(prm.addr + (size_t)idx * prm.addr_stride);
#pragma unroll
      for (int i = 0; i < 5; ++i) dst[i] = ok ? a[i] : 0u;
    }
    if (prm.pub) {
      uint8_t* dst = prm.pub + (size_t)idx * 65;
      if (ok) {
        dst[0] = 4;
        write_be32(dst + 1, X);
        write_be32(dst + 33, Y);
      } else {
        for (int i = 0; i < 65; ++i) dst[i] = 0;
      }
    }
  }
  st->mark(6);
  if (prm.ls_done) {  // host-buffer form: this workgroup's outputs are complete
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's stores acknowledged
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(prm.ls_done + (blockIdx.x - bias), prm.ls_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  if constexpr (!std::is_same<ST, NoStamp>::value) {
    if ((threadIdx.x & 63) == 0) {
      const uint32_t w = blockIdx.x * (WG / 64) + (threadIdx.x >> 6);
#pragma unroll
      for (int i = 0; i < 8; ++i) stamps[(size_t)w * 8 + i] = st_.acc[i];
    }
  }
}

#ifndef EGES_RECOVER_WAVES
#define EGES_RECOVER_WAVES 2
#endif
__global__ void __launch_bounds__(WG, EGES_RECOVER_WAVES) recover_kernel(RecoverParams prm) {
  if (prm.ls_host && blockIdx.x == 0) {
    ls_mirror(prm);
    return;
  }
  recover_body<NoStamp>(prm, nullptr);
}

#ifdef EGES_PHASE_STAMPS
__global__ void __launch_bounds__(WG, 2) recover_kernel_stamped(RecoverParams prm, uint64_t* stamps) {
  recover_body<Stamper>(prm, stamps);
}
#endif

// ------------------------------------------------------------------ launcher
hipError_t launch_recover(const RecoverParams& p, int max_blocks, int ws_blocks, hipStream_t st) {
  if (p.n == 0) return hipSuccess;
  const int grid = grid_for_lane_serial(p.n, max_blocks);
  if (grid > ws_blocks) return hipErrorInvalidValue;  // the kernel indexes ws by blockIdx.x
  hipLaunchKernelGGL(recover_kernel, dim3(grid), dim3(WG), 0, st, p);
  return hipGetLastError();
}

#ifdef EGES_PHASE_STAMPS
hipError_t launch_recover_stamped(const RecoverParams& p, int max_blocks, int ws_blocks, hipStream_t st, uint64_t* stamps) {
  if (p.n == 0) return hipSuccess;
  const int grid = grid_for_lane_serial(p.n, max_blocks);
  if (grid > ws_blocks) return hipErrorInvalidValue;
  hipLaunchKernelGGL(recover_kernel_stamped, dim3(grid), dim3(WG), 0, st, p, stamps);
  return hipGetLastError();
}
#endif

hipError_t launch_recover_host(const RecoverParams& p, int grid, int ws_blocks, hipStream_t st) {
  if (p.n == 0) return hipSuccess;
  if (!p.ls_host || grid + 1 > ws_blocks || (uint64_t)grid * WG * MAX_SLOTS < p.n) return hipErrorInvalidValue;
  hipLaunchKernelGGL(recover_kernel, dim3(grid + 1), dim3(WG), 0, st, p);
  return hipGetLastError();
}

int lane_serial_grid(uint32_t n, int max_blocks) { return grid_for_lane_serial(n, max_blocks); }

int occupancy_recover() {
  int b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, recover_kernel, WG, 0) != hipSuccess || b < 1) b = 1;
  return b;
}

}  // namespace eges
