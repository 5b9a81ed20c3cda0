#include <chrono>
#include <thread>
#include <vector>
#include <cstdio>
#include <cstdint>
int main() {
  for (int T : {1, 2, 4, 8}) {
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th; std::vector<uint64_t> out(T);
    for (int t = 0; t < T; ++t) th.emplace_back([&, t] { uint64_t x = t; for (long i = 0; i < 200000000L / T; ++i) x = x * 6364136223846793005ULL + 1; out[t] = x; });
    for (auto& x : th) x.join();
    auto t1 = std::chrono::steady_clock::now();
    printf("T=%d: %.3f ms\n", T, std::chrono::duration<double, std::milli>(t1 - t0).count());
  }
}
