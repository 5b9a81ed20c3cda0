#define OPENSSL_SUPPRESS_DEPRECATED
#include <openssl/sha.h>
#include <chrono>
#include <thread>
#include <vector>
#include <cstdio>
#include <cstdint>
int main() {
  const int N = 3840; const size_t B = 1600;
  std::vector<uint8_t> data(N * B, 7);
  for (int T : {1, 2, 4, 8, 16}) {
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back([&, t] {
      uint8_t d[32];
      for (int i = t; i < N; i += T) { SHA256_CTX c; SHA256_Init(&c); SHA256_Update(&c, data.data() + (size_t)i * B, B); SHA256_Final(d, &c); }
    });
    for (auto& x : th) x.join();
    auto t1 = std::chrono::steady_clock::now();
    printf("T=%d low-level: %.3f ms\n", T, std::chrono::duration<double, std::milli>(t1 - t0).count());
  }
}
