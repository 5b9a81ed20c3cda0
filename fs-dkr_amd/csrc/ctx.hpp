// Internal context object behind the opaque fsdkr_ctx handle.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <string>
#include <vector>

namespace fsdkr {

struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
};

struct TimeAcc {
  double ms = 0.0;
  uint32_t launches = 0;
};

struct PendingEvent {
  std::string name;
  hipEvent_t e0;
  hipEvent_t e1;
};

struct Ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool timing = false;
  std::string err;
  std::map<std::string, DevBuf> bufs;
  std::map<std::string, TimeAcc> times;
  std::vector<PendingEvent> pending;
  std::vector<uint8_t> staging;   // host staging for descriptor uploads
  static constexpr int NSIDE = 8;
  hipStream_t side[NSIDE] = {};   // concurrent streams for independent jobs (lazily created)
  void* plan = nullptr;           // prepared collect() batch (collect.cpp)

  void fail(const char* fmt, ...);
  int hip_check(hipError_t e, const char* what);
  // grow-only named device buffer (contents undefined after growth)
  void* buf(const char* name, size_t bytes);
  // HIP-event brackets around a kernel launch (timing mode only); st = nullptr: main stream
  void mark(const char* name, bool begin) { if (begin) tbeg(name, stream); else tend(last_mark, stream); }
  size_t tbeg(const char* name, hipStream_t st);
  void tend(size_t idx, hipStream_t st);
  size_t last_mark = (size_t)-1;
  hipStream_t side_stream(int k);
  // synchronise the stream and fold pending events into `times`
  int sync();
};

// A batch of modexp instances of one modulus width (k32 limbs) and one
// exponent-length class (exp_bits = max bits; sets the window count).
struct ModexpJob {
  uint32_t k32 = 0;
  uint32_t exp_bits = 0;
  std::vector<uint64_t> base_ptr, exp_ptr;   // device addresses
  std::vector<uint32_t> base_len, exp_len;   // limbs
  std::vector<uint32_t> mod_idx;
  void add(uint64_t b, uint32_t blen, uint64_t e, uint32_t elen, uint32_t ebits, uint32_t m) {
    base_ptr.push_back(b);
    base_len.push_back(blen);
    exp_ptr.push_back(e);
    exp_len.push_back(elen);
    mod_idx.push_back(m);
    if (ebits > exp_bits) exp_bits = ebits;
  }
  size_t size() const { return base_ptr.size(); }
  size_t desc_bytes() const { return size() * (8 + 8 + 4 + 4 + 4); }
  // append base_ptr | exp_ptr | base_len | exp_len | mod_idx
  void pack(std::vector<uint8_t>& dst) const;
};

uint32_t choose_window(uint32_t ebits);
void free_collect_plan(Ctx* c);
int launch_modexp_job(Ctx* c, const ModexpJob& job, const uint32_t* d_consts, uint32_t* d_out, const char* tag);
int launch_modexp_desc(Ctx* c, uint32_t k32, uint32_t count, uint32_t exp_bits, const uint8_t* d_desc,
                       const uint32_t* d_consts, uint32_t* d_out, hipStream_t st = nullptr,
                       const char* table_tag = "mxtable");
int setup_moduli(Ctx* c, uint32_t k32, const uint32_t* d_mods, uint32_t n_mod, uint32_t** d_consts, const char* tag);
int run_modexp_device(Ctx* c, uint32_t k32, uint32_t count, const uint32_t* d_base, const uint32_t* d_exp,
                      uint32_t exp_limbs, uint32_t exp_bits, const uint32_t* d_mod_idx, const uint32_t* d_mods,
                      uint32_t n_mod, uint32_t* d_out);

}  // namespace fsdkr
