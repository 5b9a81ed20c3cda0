// The host SHA-256 of the pre-passes (OpenSSL EVP, SHA-NI), fetched once.
#pragma once
#include <openssl/evp.h>

namespace fsdkr {

// EVP_sha256() makes every EVP_DigestInit_ex repeat an implicit provider fetch
// that serialises the host threads (OpenSSL 3: 3840 PDL transcripts took
// 3.1-4.5 ms on 1-16 threads; with the fetched method 2.8 ms on one thread and
// 0.6 ms on 16, tools/microbench/sha_threads.cpp on the GPU box).
inline const EVP_MD* sha256_md() {
  static const EVP_MD* md = [] {
    const EVP_MD* m = EVP_MD_fetch(nullptr, "SHA256", nullptr);
    return m ? m : EVP_sha256();
  }();
  return md;
}

}  // namespace fsdkr
