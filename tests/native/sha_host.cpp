// Host-side check of fs-dkr_amd/csrc/sha256.hpp (the same code runs on the
// device): reads little-endian u32 limb arrays from stdin as
// "<nvals> { <nlimbs> <limb>... }" and prints SHA-256(to_bytes(v0) || ...)
// as 8 little-endian limbs (BigInt::from_bytes(digest)).
#include <cstdio>
#include <vector>
#include "sha256.hpp"
int main() {
  unsigned nv;
  if (scanf("%u", &nv) != 1) return 1;
  fsdkr::Sha256 h;
  h.init();
  for (unsigned k = 0; k < nv; ++k) {
    unsigned n;
    if (scanf("%u", &n) != 1) return 1;
    std::vector<uint32_t> v(n);
    for (unsigned j = 0; j < n; ++j)
      if (scanf("%u", &v[j]) != 1) return 1;
    h.bigint(v.data(), n);
  }
  uint32_t d[8];
  h.finish_le(d);
  for (int i = 0; i < 8; ++i) printf("%u ", d[i]);
  printf("\n");
  return 0;
}
