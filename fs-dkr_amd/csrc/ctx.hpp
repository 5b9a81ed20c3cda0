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

  void fail(const char* fmt, ...);
  int hip_check(hipError_t e, const char* what);
  // grow-only named device buffer (contents undefined after growth)
  void* buf(const char* name, size_t bytes);
  // HIP-event brackets around a kernel launch on `stream` (timing mode only)
  void mark(const char* name, bool begin);
  // synchronise the stream and fold pending events into `times`
  int sync();
};

uint32_t choose_window(uint32_t ebits);
int run_modexp_device(Ctx* c, uint32_t k32, uint32_t count, const uint32_t* d_base, const uint32_t* d_exp,
                      uint32_t exp_limbs, uint32_t exp_bits, const uint32_t* d_mod_idx, const uint32_t* d_mods,
                      uint32_t n_mod, uint32_t* d_out);

}  // namespace fsdkr
