// Host-side check of hbn::SmallFactorSieve (fs-dkr_amd/csrc/hostbn.hpp, the
// correct-key primorial check in prepare): reads "<count> { <nlimbs> <limb>... }"
// little-endian u32 limb arrays from stdin and prints, per value, the sieve's
// answer and the round-2 has_small_factor's (primes below 6370, as collect.hpp).
#include <cstdio>
#include <vector>
#include "hostbn.hpp"
int main() {
  std::vector<uint32_t> primes;
  std::vector<bool> comp(6370, false);
  for (uint32_t i = 2; i < 6370; ++i) {
    if (comp[i]) continue;
    primes.push_back(i);
    for (uint32_t j = i * i; j < 6370; j += i) comp[j] = true;
  }
  const fsdkr::hbn::SmallFactorSieve sv(primes, 192);
  unsigned cnt;
  if (scanf("%u", &cnt) != 1) return 1;
  for (unsigned k = 0; k < cnt; ++k) {
    unsigned n;
    if (scanf("%u", &n) != 1 || n > 192) return 1;
    std::vector<uint32_t> v(n);
    for (unsigned j = 0; j < n; ++j)
      if (scanf("%u", &v[j]) != 1) return 1;
    printf("%d %d\n", sv.divides(v.data(), n) ? 1 : 0, fsdkr::hbn::has_small_factor(v.data(), n, primes) ? 1 : 0);
  }
  return 0;
}
