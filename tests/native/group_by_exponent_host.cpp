// Host-side check of group_by_exponent (fs-dkr_amd/csrc/ctx.hpp): the regrouping
// of a modexp job so every wave's instances share their exponent (GA
// receiver-major, job 1).  Reads "<per_wave> <pad_row> <count> { <exp_key>
// <exp_len> }" and prints the aligned flag, then one line per output instance:
// "<source instance> <out row> <exp key>".
#include <cstdio>
#include "ctx.hpp"
int main() {
  unsigned per_wave, pad, cnt;
  if (scanf("%u %u %u", &per_wave, &pad, &cnt) != 3) return 1;
  fsdkr::ModexpJob J;
  J.k32 = 128;
  for (unsigned k = 0; k < cnt; ++k) {
    unsigned long long key;
    unsigned elen;
    if (scanf("%llu %u", &key, &elen) != 2) return 1;
    // the base address encodes the source instance
    J.add(0x100000ull + 16ull * k, 128, key, elen, 32 * elen, k % 7);
  }
  const bool aligned = fsdkr::group_by_exponent(J, per_wave, pad);
  printf("%d\n", aligned ? 1 : 0);
  for (size_t i = 0; i < J.size(); ++i)
    printf("%llu %u %llu\n", (unsigned long long)((J.base_ptr[i] - 0x100000ull) / 16), J.out_idx[i],
           (unsigned long long)J.exp_ptr[i]);
  return 0;
}
