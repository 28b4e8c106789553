// ThreadSanitizer driver of csrc/copy_pool.hpp (the host-buffer path's split staging memcpy,
// tests/test_sanitizers.py): several caller threads, as several contexts' host calls would, copy
// blocks of varied sizes with varied thread counts through the one process-wide pool at once, and
// every destination is checked byte for byte.  Any data race or lost wake-up fails the run (TSan
// report, or the 60 s alarm of a hang).
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <thread>
#include <vector>

#include "copy_pool.hpp"

int main(int argc, char **argv) {
  alarm(60);
  const int callers = argc > 1 ? atoi(argv[1]) : 4;
  const int rounds = argc > 2 ? atoi(argv[2]) : 40;
  std::atomic<int> bad{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < callers; t++) {
    ts.emplace_back([t, rounds, &bad] {
      unsigned seed = 0x9E3779B9u * (t + 1);
      auto rnd = [&seed] { return seed = seed * 1664525u + 1013904223u; };
      for (int r = 0; r < rounds; r++) {
        // below one part (plain memcpy), a few parts, and a size that is not a multiple of the
        // 4 KiB step rounding
        const size_t sizes[] = {4096, (size_t)3 << 20, ((size_t)5 << 20) + 12345, (size_t)9 << 20};
        const size_t bytes = sizes[rnd() % 4];
        const unsigned threads = 1 + rnd() % 12;
        std::vector<unsigned char> src(bytes), dst(bytes, 0xEE);
        for (size_t i = 0; i < bytes; i++) src[i] = (unsigned char)(i * 131 + r * 7 + t);
        nttmul::CopyPool::get().copy(dst.data(), src.data(), bytes, threads);
        if (memcmp(dst.data(), src.data(), bytes) != 0) bad++;
      }
    });
  }
  for (auto &th : ts) th.join();
  if (bad) {
    printf("copy pool: %d mismatching copies\n", bad.load());
    return 1;
  }
  printf("copy pool tsan run ok (%d callers x %d copies)\n", callers, rounds);
  return 0;
}
