// capi.cpp — C ABI (include/qpgpu.h) over the gfx950 kernels: contexts,
// PolynomialBatch commitments, openings and primitives.
#include "../../include/qpgpu.h"
#include <string.h>
#include <new>
#include "ctx.h"
#include "field.h"
#include "kernels.h"

extern "C" {

const char *qp_version(void) { return "qpgpu 0.1 gfx950 (MI355X)"; }

int qp_ctx_create(int device, qp_ctx **out) {
  if (!out) return QP_ERR_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) return QP_ERR_HIP;
  qp_ctx *c = new (std::nothrow) qp_ctx();
  if (!c) return QP_ERR_OOM;
  c->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return QP_ERR_HIP;
  }
  c->stream = c->own_stream;
  if (qpk::twiddles_init(c->tw, c->stream) != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess) {
    qpk::twiddles_free(c->tw);
    (void)hipStreamDestroy(c->own_stream);
    delete c;
    return QP_ERR_HIP;
  }
  *out = c;
  return QP_OK;
}

void qp_ctx_destroy(qp_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  qpk::twiddles_free(c->tw);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
}

const char *qp_ctx_last_error(const qp_ctx *c) { return c ? c->err.c_str() : "null context"; }

int qp_ctx_set_stream(qp_ctx *c, void *s) {
  if (!c) return QP_ERR_ARG;
  c->stream = s ? (hipStream_t)s : c->own_stream;
  return QP_OK;
}

// the context's own stream re-created at the device's greatest (high != 0) or
// default priority: the aggregation levels' latency-bound launches then
// dispatch ahead of leaf-proof kernels queued on normal-priority streams
int qp_ctx_set_priority(qp_ctx *c, int high) {
  if (!c) return QP_ERR_ARG;
  QP_HIP_TRY(c, hipSetDevice(c->device));
  int least = 0, greatest = 0;
  QP_HIP_TRY(c, hipDeviceGetStreamPriorityRange(&least, &greatest));
  hipStream_t s = nullptr;
  QP_HIP_TRY(c, hipStreamCreateWithPriority(&s, hipStreamNonBlocking, high ? greatest : least));
  QP_HIP_TRY(c, hipStreamSynchronize(c->own_stream));
  const bool own = c->stream == c->own_stream;
  (void)hipStreamDestroy(c->own_stream);
  c->own_stream = s;
  if (own) c->stream = s;
  return QP_OK;
}

int qp_ctx_synchronize(qp_ctx *c) {
  if (!c) return QP_ERR_ARG;
  QP_HIP_TRY(c, hipStreamSynchronize(c->stream));
  return QP_OK;
}

static int check_shape(qp_ctx *c, uint32_t npolys, uint32_t log_n, uint32_t rate_bits, uint32_t cap_h) {
  if (!c) return QP_ERR_ARG;
  if (npolys == 0 || log_n > qpk::BIG_LOG_MAX || rate_bits > 6 || log_n + rate_bits > qpk::TW_LOG ||
      cap_h > log_n + rate_bits) {
    c->err = "unsupported shape (need log_n <= 16, log_n + rate_bits <= 18, cap_h <= log N)";
    return QP_ERR_ARG;
  }
  return QP_OK;
}

void qp_batch_free(qp_batch *b) {
  if (!b) return;
  if (b->d_coeffs) (void)hipFree(b->d_coeffs);
  if (b->d_lde) (void)hipFree(b->d_lde);
  if (b->d_salt) (void)hipFree(b->d_salt);
  if (b->d_dig) (void)hipFree(b->d_dig);
  delete b;
}

static int batch_alloc(qp_ctx *c, uint32_t nbat, uint32_t npolys, uint32_t log_n, uint32_t rate_bits, uint32_t cap_h,
                       uint32_t nsalt, qp_batch **out) {
  qp_batch *b = new (std::nothrow) qp_batch();
  if (!b) return QP_ERR_OOM;
  b->ctx = c; b->nbat = nbat; b->npolys = npolys; b->nsalt = nsalt;
  b->log_n = log_n; b->rate_bits = rate_bits; b->cap_h = cap_h;
  hipError_t e = hipMalloc(&b->d_coeffs, (size_t)nbat * npolys * b->n() * 8);
  if (!e) e = hipMalloc(&b->d_lde, (size_t)nbat * npolys * b->N() * 8);
  if (!e && nsalt) e = hipMalloc(&b->d_salt, (size_t)nbat * b->N() * nsalt * 8);
  if (!e) e = hipMalloc(&b->d_dig, (size_t)nbat * b->ndig() * 32);
  if (e) {
    c->err = std::string("batch alloc: ") + hipGetErrorString(e);
    qp_batch_free(b);
    return QP_ERR_OOM;
  }
  *out = b;
  return QP_OK;
}

// LDE + leaves + tree for a batch whose d_coeffs are filled
static void batch_build(qp_batch *b) {
  qp_ctx *c = b->ctx;
  const uint64_t n = b->n(), N = b->N();
  const uint32_t logN = b->log_n + b->rate_bits;
  qpk::lde(c->tw, b->d_coeffs, n, b->d_lde, N, b->npolys, b->log_n, b->rate_bits, gl::GEN, b->nbat,
           (uint64_t)b->npolys * n, (uint64_t)b->npolys * N, c->stream);
  qpk::leaf_hash_tree(b->d_lde, N, b->npolys, b->d_salt, b->nsalt, b->d_dig, logN, b->cap_h, b->nbat,
                      (uint64_t)b->npolys * N, N * b->nsalt, b->ndig() * 4, c->stream);
}

static uint64_t *cap_ptr(qp_batch *b, uint32_t bi) {
  const uint32_t logN = b->log_n + b->rate_bits;
  return b->d_dig + bi * b->ndig() * 4 + qpk::tree_level_offset(logN, logN - b->cap_h) * 4;
}

static int commit_common(qp_ctx *c, const uint64_t *host_in, bool from_coeffs, uint32_t npolys, uint32_t log_n,
                         uint32_t rate_bits, uint32_t cap_h, const uint64_t *salt, uint32_t nsalt,
                         uint64_t *coeffs_out, uint64_t *cap_out, qp_batch **out) {
  int st = check_shape(c, npolys, log_n, rate_bits, cap_h);
  if (st) return st;
  if (!host_in || !cap_out || (nsalt && !salt)) { c->err = "null argument"; return QP_ERR_ARG; }
  QP_HIP_TRY(c, hipSetDevice(c->device));
  qp_batch *b = nullptr;
  st = batch_alloc(c, 1, npolys, log_n, rate_bits, cap_h, nsalt, &b);
  if (st) return st;
  const uint64_t n = b->n(), N = b->N();
  hipError_t e = hipSuccess;
  if (from_coeffs) {
    e = hipMemcpyAsync(b->d_coeffs, host_in, npolys * n * 8, hipMemcpyHostToDevice, c->stream);
  } else {
    // values land in the LDE buffer (scratch), ifft into d_coeffs
    e = hipMemcpyAsync(b->d_lde, host_in, npolys * n * 8, hipMemcpyHostToDevice, c->stream);
    if (!e) qpk::intt(c->tw, b->d_lde, n, b->d_coeffs, n, npolys, log_n, 1, 0, 0, c->stream);
  }
  if (!e && nsalt) e = hipMemcpyAsync(b->d_salt, salt, N * nsalt * 8, hipMemcpyHostToDevice, c->stream);
  if (!e) {
    batch_build(b);
    e = hipGetLastError();
  }
  if (!e && coeffs_out) e = hipMemcpyAsync(coeffs_out, b->d_coeffs, npolys * n * 8, hipMemcpyDeviceToHost, c->stream);
  if (!e) e = hipMemcpyAsync(cap_out, cap_ptr(b, 0), ((size_t)32 << cap_h), hipMemcpyDeviceToHost, c->stream);
  if (!e) e = hipStreamSynchronize(c->stream);
  if (e) {
    c->err = std::string("commit: ") + hipGetErrorString(e);
    qp_batch_free(b);
    return QP_ERR_HIP;
  }
  if (out) *out = b;
  else qp_batch_free(b);
  return QP_OK;
}

int qp_commit_values(qp_ctx *c, const uint64_t *values, uint32_t npolys, uint32_t log_n, uint32_t rate_bits,
                     uint32_t cap_h, const uint64_t *salt, uint32_t nsalt, uint64_t *coeffs_out, uint64_t *cap_out,
                     qp_batch **out) {
  return commit_common(c, values, false, npolys, log_n, rate_bits, cap_h, salt, nsalt, coeffs_out, cap_out, out);
}

int qp_commit_coeffs(qp_ctx *c, const uint64_t *coeffs, uint32_t npolys, uint32_t log_n, uint32_t rate_bits,
                     uint32_t cap_h, const uint64_t *salt, uint32_t nsalt, uint64_t *cap_out, qp_batch **out) {
  return commit_common(c, coeffs, true, npolys, log_n, rate_bits, cap_h, salt, nsalt, nullptr, cap_out, out);
}

int qp_commit_values_dev(qp_ctx *c, const uint64_t *d_values, uint32_t nbat, uint32_t npolys, uint32_t log_n,
                         uint32_t rate_bits, uint32_t cap_h, uint64_t *d_cap_out, qp_batch **out) {
  int st = check_shape(c, npolys, log_n, rate_bits, cap_h);
  if (st) return st;
  if (!d_values || !out || !nbat) { c->err = "null argument"; return QP_ERR_ARG; }
  qp_batch *b = *out;
  if (b && (b->nbat != nbat || b->npolys != npolys || b->log_n != log_n || b->rate_bits != rate_bits ||
            b->cap_h != cap_h || b->nsalt)) {
    c->err = "reused batch handle has a different shape";
    return QP_ERR_ARG;
  }
  if (!b) {
    st = batch_alloc(c, nbat, npolys, log_n, rate_bits, cap_h, 0, &b);
    if (st) return st;
    *out = b;
  }
  const uint64_t n = b->n();
  qpk::intt(c->tw, d_values, n, b->d_coeffs, n, npolys, log_n, nbat, (uint64_t)npolys * n, (uint64_t)npolys * n,
            c->stream);
  batch_build(b);
  if (d_cap_out)
    for (uint32_t bi = 0; bi < nbat; bi++)
      QP_HIP_TRY(c, hipMemcpyAsync(d_cap_out + (size_t)bi * (4u << cap_h), cap_ptr(b, bi), (size_t)32 << cap_h,
                                   hipMemcpyDeviceToDevice, c->stream));
  QP_HIP_TRY(c, hipGetLastError());
  return QP_OK;
}

int qp_batch_open(qp_batch *b, const uint32_t *idx, uint32_t nidx, uint64_t *leaves_out, uint64_t *sib_out) {
  if (!b) return QP_ERR_ARG;
  qp_ctx *c = b->ctx;
  const uint64_t N = b->N();
  const uint32_t logN = b->log_n + b->rate_bits, W = b->npolys + b->nsalt, depth = logN - b->cap_h;
  for (uint32_t q = 0; q < nidx; q++)
    if (idx[q] >= N) { c->err = "leaf index out of range"; return QP_ERR_ARG; }
  uint32_t *d_idx = nullptr;
  uint64_t *d_rows = nullptr, *d_sib = nullptr;
  QP_HIP_TRY(c, hipMalloc(&d_idx, nidx * 4ull + 4));
  QP_HIP_TRY(c, hipMalloc(&d_rows, (size_t)nidx * W * 8 + 8));
  QP_HIP_TRY(c, hipMalloc(&d_sib, (size_t)nidx * depth * 32 + 8));
  QP_HIP_TRY(c, hipMemcpyAsync(d_idx, idx, nidx * 4ull, hipMemcpyHostToDevice, c->stream));
  qpk::gather_rows(b->d_lde, N, b->npolys, d_idx, nidx, d_rows, c->stream);
  qpk::gather_paths(b->d_dig, logN, b->cap_h, d_idx, nidx, d_sib, c->stream);
  QP_HIP_TRY(c, hipGetLastError());
  uint64_t *tmp = new uint64_t[(size_t)nidx * b->npolys + 1];
  QP_HIP_TRY(c, hipMemcpyAsync(tmp, d_rows, (size_t)nidx * b->npolys * 8, hipMemcpyDeviceToHost, c->stream));
  if (sib_out) QP_HIP_TRY(c, hipMemcpyAsync(sib_out, d_sib, (size_t)nidx * depth * 32, hipMemcpyDeviceToHost, c->stream));
  hipError_t e = hipStreamSynchronize(c->stream);
  if (!e && leaves_out) {
    for (uint32_t q = 0; q < nidx; q++) {
      memcpy(leaves_out + (size_t)q * W, tmp + (size_t)q * b->npolys, b->npolys * 8ull);
      if (b->nsalt)
        e = hipMemcpy(leaves_out + (size_t)q * W + b->npolys, b->d_salt + (size_t)idx[q] * b->nsalt, b->nsalt * 8ull,
                      hipMemcpyDeviceToHost);
    }
  }
  delete[] tmp;
  (void)hipFree(d_idx); (void)hipFree(d_rows); (void)hipFree(d_sib);
  QP_HIP_TRY(c, e);
  return QP_OK;
}

int qp_batch_lde(qp_batch *b, uint64_t *out) {
  if (!b || !out) return QP_ERR_ARG;
  QP_HIP_TRY(b->ctx, hipMemcpy(out, b->d_lde, (size_t)b->nbat * b->npolys * b->N() * 8, hipMemcpyDeviceToHost));
  return QP_OK;
}

int qp_batch_coeffs(qp_batch *b, uint64_t *out) {
  if (!b || !out) return QP_ERR_ARG;
  QP_HIP_TRY(b->ctx, hipMemcpy(out, b->d_coeffs, (size_t)b->nbat * b->npolys * b->n() * 8, hipMemcpyDeviceToHost));
  return QP_OK;
}

int qp_ifft(qp_ctx *c, uint64_t *data, uint32_t ncols, uint32_t log_n) {
  int st = check_shape(c, ncols, log_n, 0, 0);
  if (st) return st;
  const size_t bytes = (size_t)ncols * 8 << log_n;
  uint64_t *d = nullptr, *d2 = nullptr;
  QP_HIP_TRY(c, hipMalloc(&d, bytes));
  QP_HIP_TRY(c, hipMalloc(&d2, bytes));
  QP_HIP_TRY(c, hipMemcpyAsync(d, data, bytes, hipMemcpyHostToDevice, c->stream));
  qpk::intt(c->tw, d, 1ull << log_n, d2, 1ull << log_n, ncols, log_n, 1, 0, 0, c->stream);
  QP_HIP_TRY(c, hipMemcpyAsync(data, d2, bytes, hipMemcpyDeviceToHost, c->stream));
  QP_HIP_TRY(c, hipStreamSynchronize(c->stream));
  (void)hipFree(d); (void)hipFree(d2);
  return QP_OK;
}

int qp_lde(qp_ctx *c, const uint64_t *coeffs, uint32_t ncols, uint32_t log_n, uint32_t rate_bits, uint64_t shift,
           uint64_t *out) {
  int st = check_shape(c, ncols, log_n, rate_bits, 0);
  if (st) return st;
  const uint64_t n = 1ull << log_n, N = n << rate_bits;
  uint64_t *d = nullptr, *d2 = nullptr;
  QP_HIP_TRY(c, hipMalloc(&d, ncols * n * 8));
  QP_HIP_TRY(c, hipMalloc(&d2, ncols * N * 8));
  QP_HIP_TRY(c, hipMemcpyAsync(d, coeffs, ncols * n * 8, hipMemcpyHostToDevice, c->stream));
  qpk::lde(c->tw, d, n, d2, N, ncols, log_n, rate_bits, shift, 1, 0, 0, c->stream);
  QP_HIP_TRY(c, hipMemcpyAsync(out, d2, ncols * N * 8, hipMemcpyDeviceToHost, c->stream));
  QP_HIP_TRY(c, hipStreamSynchronize(c->stream));
  (void)hipFree(d); (void)hipFree(d2);
  return QP_OK;
}

int qp_poseidon_permute(qp_ctx *c, uint64_t *states, uint64_t n) {
  if (!c || (!states && n)) return QP_ERR_ARG;
  if (!n) return QP_OK;
  uint64_t *d = nullptr;
  QP_HIP_TRY(c, hipMalloc(&d, n * 96));
  QP_HIP_TRY(c, hipMemcpyAsync(d, states, n * 96, hipMemcpyHostToDevice, c->stream));
  qpk::permute_batch(d, n, c->stream);
  QP_HIP_TRY(c, hipMemcpyAsync(states, d, n * 96, hipMemcpyDeviceToHost, c->stream));
  QP_HIP_TRY(c, hipStreamSynchronize(c->stream));
  (void)hipFree(d);
  return QP_OK;
}

}  // extern "C"
