// host_util.h — host-side Challenger (plonky2 iop/challenger.rs, SURVEY.md
// A.4), a small thread pool for per-proof host work, and a byte writer.
#pragma once
#include <stdint.h>
#include <string.h>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>
#include "field.h"
#include "poseidon.h"

namespace qh {

// duplex sponge, rate 8: observe -> input buffer (duplex at 8); get pops the
// LAST of state[0..8], duplexing first if input is pending or output empty
struct Challenger {
  uint64_t state[12] = {0};
  uint64_t in[8];
  uint32_t nin = 0;
  uint64_t out[8];
  uint32_t nout = 0;
  void duplex() {
    for (uint32_t i = 0; i < nin; i++) state[i] = in[i];
    nin = 0;
    ps::permute(state);
    memcpy(out, state, 64);
    nout = 8;
  }
  void observe(uint64_t x) {
    nout = 0;
    in[nin++] = x;
    if (nin == 8) duplex();
  }
  void observe(const uint64_t *x, size_t n) {
    for (size_t i = 0; i < n; i++) observe(x[i]);
  }
  uint64_t get() {
    if (nin || !nout) duplex();
    return out[--nout];
  }
  gl::ext get_ext() {
    uint64_t a = get();
    uint64_t b = get();
    return gl::ext{a, b};
  }
};

inline void hash_no_pad(const uint64_t *in, size_t n, uint64_t out[4]) {
  uint64_t s[12] = {0};
  for (size_t off = 0; off < n; off += 8) {
    for (size_t i = 0; i < 8 && off + i < n; i++) s[i] = in[off + i];
    ps::permute(s);
  }
  memcpy(out, s, 32);
}

// hash_n_to_m_with_pad(input || 1 || 0* || 1)
inline void hash_pad(const uint64_t *in, size_t n, uint64_t out[4]) {
  std::vector<uint64_t> v(in, in + n);
  v.push_back(1);
  while ((v.size() + 1) % 8) v.push_back(0);
  v.push_back(1);
  hash_no_pad(v.data(), v.size(), out);
}

class ThreadPool {
 public:
  explicit ThreadPool(unsigned n) {
    for (unsigned i = 0; i < n; i++) workers_.emplace_back([this] { loop(); });
  }
  ~ThreadPool() {
    {
      std::lock_guard<std::mutex> l(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : workers_) t.join();
  }
  // runs f(i) for i in [0, n) on the pool and the caller; returns when done
  void parallel_for(size_t n, const std::function<void(size_t)> &f) {
    if (n == 0) return;
    if (workers_.empty() || n == 1) {
      for (size_t i = 0; i < n; i++) f(i);
      return;
    }
    std::atomic<size_t> next{0};
    auto body = [&] {
      size_t i;
      while ((i = next.fetch_add(1)) < n) f(i);
    };
    {
      std::lock_guard<std::mutex> l(m_);
      job_ = body;
      gen_++;
    }
    cv_.notify_all();
    body();
    // close the job, then wait for every worker that entered it to leave
    std::unique_lock<std::mutex> l(m_);
    job_ = nullptr;
    idle_cv_.wait(l, [&] { return active_ == 0; });
  }
  size_t size() const { return workers_.size(); }

 private:
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return stop_ || (gen_ != seen && job_); });
        if (stop_) return;
        seen = gen_;
        job = job_;
        active_++;
      }
      job();
      {
        std::lock_guard<std::mutex> l(m_);
        active_--;
      }
      idle_cv_.notify_all();
    }
  }
  std::vector<std::thread> workers_;
  std::mutex m_;
  std::condition_variable cv_, idle_cv_;
  unsigned active_ = 0;
  std::function<void()> job_;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

struct ByteWriter {
  uint8_t *p;
  size_t pos = 0;
  explicit ByteWriter(uint8_t *dst) : p(dst) {}
  void u64(uint64_t v) {
    if (p) memcpy(p + pos, &v, 8);
    pos += 8;
  }
  void u8(uint8_t v) {
    if (p) p[pos] = v;
    pos += 1;
  }
  void u64s(const uint64_t *v, size_t n) {
    if (p) memcpy(p + pos, v, 8 * n);
    pos += 8 * n;
  }
};

}  // namespace qh
