// ctx.h — internal definitions behind the C ABI handles (qpgpu.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include "kernels.h"

struct qp_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  qpk::Twiddles tw;
  std::string err;
};

struct qp_batch {
  qp_ctx *ctx = nullptr;
  uint32_t nbat = 1, npolys = 0, nsalt = 0, log_n = 0, rate_bits = 0, cap_h = 0;
  uint64_t *d_coeffs = nullptr;  // [nbat][npolys][n]
  uint64_t *d_lde = nullptr;     // [nbat][npolys][N] leaf order
  uint64_t *d_salt = nullptr;    // [nbat][N][nsalt]
  uint64_t *d_dig = nullptr;     // [nbat][tree digests][4]
  uint64_t n() const { return (uint64_t)1 << log_n; }
  uint64_t N() const { return (uint64_t)1 << (log_n + rate_bits); }
  uint64_t ndig() const { return qpk::tree_digest_count(log_n + rate_bits, cap_h); }
};

#define QP_HIP_TRY(ctx, expr)                                                    \
  do {                                                                           \
    hipError_t _e = (expr);                                                      \
    if (_e != hipSuccess) {                                                      \
      (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(_e);            \
      return _e == hipErrorOutOfMemory ? QP_ERR_OOM : QP_ERR_HIP;                \
    }                                                                            \
  } while (0)
