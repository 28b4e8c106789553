// copy_pool.hpp — the host-buffer path's staging memcpy split over a few host threads
// (csrc/nttmul.cpp pcopy).  Header-only and free of HIP so that tests/sanitize/tsan_copy_pool.cpp
// can drive it under ThreadSanitizer (tests/test_sanitizers.py).
#pragma once
#include <algorithm>
#include <condition_variable>
#include <cstddef>
#include <cstring>
#include <mutex>
#include <thread>

namespace nttmul {

// memcpy split over a few host threads for large blocks (the staging copies bound the
// host-buffer path: one core moves ~10-20 GB/s, a PCIe Gen5 x16 link ~50 GB/s each way).  The
// workers are started once and live for the process (never joined: the pool is never freed).
constexpr unsigned kMaxCopyThreads = 64;
class CopyPool {
 public:
  static CopyPool &get() {
    static CopyPool *pool = new CopyPool();
    return *pool;
  }
  // split over at most `threads` threads (the caller's included)
  void copy(void *dst, const void *src, size_t bytes, unsigned threads) {
    const size_t kPart = 1u << 20;
    size_t parts = std::min<size_t>(std::min<size_t>(cap_, threads), bytes / kPart);
    if (parts <= 1) {
      memcpy(dst, src, bytes);
      return;
    }
    std::unique_lock<std::mutex> call(call_mu_);  // one split copy at a time
    parts = std::min<size_t>(parts, grow((unsigned)parts - 1) + 1);
    if (parts <= 1) {
      memcpy(dst, src, bytes);
      return;
    }
    const size_t step = (bytes / parts + 4095) & ~(size_t)4095;
    {
      std::lock_guard<std::mutex> l(mu_);
      d_ = (char *)dst;
      s_ = (const char *)src;
      bytes_ = bytes;
      step_ = step;
      pending_ = parts - 1;
      for (size_t i = 0; i + 1 < parts; i++) w_[i].go = true;
    }
    // wake exactly the workers this copy uses (each waits on its own condition variable)
    for (size_t i = 0; i + 1 < parts; i++) w_[i].cv.notify_one();
    memcpy(dst, src, std::min(step, bytes));
    std::unique_lock<std::mutex> l(mu_);
    done_.wait(l, [&] { return pending_ == 0; });
  }

 private:
  struct Worker {
    std::condition_variable cv;
    bool go = false;
  };
  CopyPool() {
    const unsigned hw = std::thread::hardware_concurrency();
    cap_ = std::min(kMaxCopyThreads, std::max(hw, 1u));
  }
  // Workers start on first use, up to the largest split any context has asked for (advisor r4:
  // not min(64, hardware threads) - 1 of them up front); returns how many are running.
  unsigned grow(unsigned want) {
    while (started_ < want && started_ + 1 < kMaxCopyThreads) {
      try {
        const unsigned i = started_;
        std::thread([this, i] { run(i); }).detach();
        started_++;
      } catch (...) {  // no thread available: split over the ones running
        break;
      }
    }
    return std::min(started_, want);
  }
  void run(unsigned i) {
    std::unique_lock<std::mutex> l(mu_);
    for (;;) {
      w_[i].cv.wait(l, [&] { return w_[i].go; });
      w_[i].go = false;
      const size_t o = (i + 1) * step_;
      char *d = d_;
      const char *s = s_;
      const size_t len = o < bytes_ ? std::min(step_, bytes_ - o) : 0;
      l.unlock();
      if (len) memcpy(d + o, s + o, len);
      l.lock();
      if (--pending_ == 0) done_.notify_one();
    }
  }
  Worker w_[kMaxCopyThreads];
  unsigned cap_ = 1, started_ = 0;  // started_: guarded by call_mu_
  std::mutex call_mu_, mu_;
  std::condition_variable done_;
  size_t pending_ = 0, bytes_ = 0, step_ = 0;
  char *d_ = nullptr;
  const char *s_ = nullptr;
};

}  // namespace nttmul
