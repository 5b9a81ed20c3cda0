#include <openssl/evp.h>
#include <chrono>
#include <thread>
#include <vector>
#include <cstdio>
#include <cstdint>
int main() {
  const int N = 3840; const size_t B = 1600;
  std::vector<uint8_t> data(N * B, 7);
  EVP_MD* fetched = EVP_MD_fetch(nullptr, "SHA256", nullptr);
  for (int T : {1, 2, 4, 8, 16}) for (int mode = 0; mode < 2; ++mode) {
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back([&, t] {
      EVP_MD_CTX* c = EVP_MD_CTX_new(); uint8_t d[32]; unsigned len;
      for (int i = t; i < N; i += T) {
        EVP_DigestInit_ex(c, mode ? fetched : EVP_sha256(), nullptr); EVP_DigestUpdate(c, data.data() + (size_t)i * B, B); EVP_DigestFinal_ex(c, d, &len);
      }
      EVP_MD_CTX_free(c);
    });
    for (auto& x : th) x.join();
    auto t1 = std::chrono::steady_clock::now();
    printf("T=%d mode %d: %.3f ms\n", T, mode, std::chrono::duration<double, std::milli>(t1 - t0).count());
  }
}
