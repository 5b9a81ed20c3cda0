// C ABI implementation (include/fsdkr/fsdkr.h): context, device buffers,
// kernel launch sequencing and per-kernel HIP-event timing.
#include "fsdkr/fsdkr.h"

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <map>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "ctx.hpp"
#include "kernels.h"
#include "verify.h"

using namespace fsdkr;

// ------------------------------------------------------------------ context ---
namespace fsdkr {

void Ctx::fail(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  err = buf;
}

int Ctx::hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return FSDKR_OK;
  fail("%s: %s", what, hipGetErrorString(e));
  if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return FSDKR_E_OOM;
  return FSDKR_E_HIP;
}

void* Ctx::buf(const char* name, size_t bytes) {
  DevBuf& b = bufs[name];
  if (b.bytes >= bytes && b.ptr) return b.ptr;
  if (b.ptr) (void)hipFree(b.ptr);
  b.ptr = nullptr;
  b.bytes = 0;
  size_t want = bytes < 256 ? 256 : bytes;
  if (hipMalloc(&b.ptr, want) != hipSuccess) {
    b.ptr = nullptr;
    return nullptr;
  }
  b.bytes = want;
  return b.ptr;
}

uint8_t* Ctx::host_arena(size_t bytes) {
  if (pinned && pinned_bytes >= bytes) return pinned;
  if (pinned) (void)hipHostFree(pinned);
  pinned = nullptr;
  pinned_bytes = 0;
  const size_t want = bytes + bytes / 4 + (1u << 20);
  if (hipHostMalloc((void**)&pinned, want, hipHostMallocDefault) != hipSuccess) {
    pinned = nullptr;
    return nullptr;
  }
  pinned_bytes = want;
  return pinned;
}

uint8_t* Ctx::host_buf(const char* name, size_t bytes) {
  DevBuf& b = hbufs[name];
  if (b.bytes >= bytes && b.ptr) return (uint8_t*)b.ptr;
  if (b.ptr) (void)hipHostFree(b.ptr);
  b.ptr = nullptr;
  b.bytes = 0;
  const size_t want = bytes + bytes / 4 + (1u << 20);
  if (hipHostMalloc(&b.ptr, want, hipHostMallocDefault) != hipSuccess) {
    b.ptr = nullptr;
    return nullptr;
  }
  b.bytes = want;
  return (uint8_t*)b.ptr;
}

static hipStream_t make_stream(const Ctx* c, int masked);

hipStream_t Ctx::aux_stream() {
  if (!aux) aux = make_stream(this, ga_cus ? 4 : 0);
  return aux ? aux : stream;
}

unsigned host_threads() {
  static unsigned n = [] {
    for (const char* k : {"FSDKR_HOST_THREADS", "OMP_NUM_THREADS"})
      if (const char* e = getenv(k)) {
        const int v = atoi(e);
        if (v > 0) return (unsigned)std::min(v, 64);
      }
    const unsigned hw = std::thread::hardware_concurrency();
    return hw ? std::min(hw, 16u) : 4u;
  }();
  return n;
}

namespace {
thread_local bool tl_pool_worker = false;

struct PoolJob {
  void (*fn)(void*, size_t);
  void* arg;
  size_t chunks;
  std::atomic<size_t> next{0};
  size_t done = 0;   // chunks finished (under the pool mutex)
  int active = 0;    // workers holding the job (under the pool mutex)
};

// Parked workers: a run publishes its job under the mutex and bumps the
// generation; every worker takes chunks until none is left, then reports them.
// The job lives on the caller's stack until every chunk is done and no worker
// holds it.
struct HostPool {
  std::mutex run_m;   // one run at a time
  std::mutex m;
  std::condition_variable cv, done_cv;
  PoolJob* cur = nullptr;
  uint64_t gen = 0;

  explicit HostPool(unsigned workers) {
    for (unsigned k = 0; k < workers; ++k) std::thread([this] { loop(); }).detach();
  }
  static size_t drain(PoolJob& j) {
    size_t did = 0;
    for (;;) {
      const size_t c = j.next.fetch_add(1);
      if (c >= j.chunks) return did;
      j.fn(j.arg, c);
      ++did;
    }
  }
  void loop() {
    tl_pool_worker = true;
    uint64_t seen = 0;
    for (;;) {
      PoolJob* j;
      {
        std::unique_lock<std::mutex> l(m);
        cv.wait(l, [&] { return gen != seen && cur != nullptr; });
        seen = gen;
        j = cur;
        ++j->active;
      }
      const size_t did = drain(*j);
      {
        std::lock_guard<std::mutex> l(m);
        j->done += did;
        --j->active;
      }
      done_cv.notify_all();
    }
  }
  void run(PoolJob& j) {
    {
      std::lock_guard<std::mutex> l(m);
      cur = &j;
      ++gen;
    }
    cv.notify_all();
    const size_t did = drain(j);
    std::unique_lock<std::mutex> l(m);
    j.done += did;
    done_cv.wait(l, [&] { return j.done == j.chunks && j.active == 0; });
    cur = nullptr;
  }
};

HostPool& host_pool() {
  static HostPool* p = new HostPool(host_threads() > 1 ? host_threads() - 1 : 0);   // never destroyed: workers parked
  return *p;
}
}  // namespace

void host_pool_run(size_t chunks, void (*fn)(void*, size_t), void* arg) {
  if (chunks == 0) return;
  if (chunks == 1) {
    fn(arg, 0);
    return;
  }
  HostPool& p = host_pool();
  std::unique_lock<std::mutex> busy(p.run_m, std::defer_lock);
  if (tl_pool_worker || !busy.try_lock()) {   // nested or concurrent: fresh threads
    std::vector<std::thread> th;
    for (size_t c = 1; c < chunks; ++c) th.emplace_back([=] { fn(arg, c); });
    fn(arg, 0);
    for (auto& t : th) t.join();
    return;
  }
  PoolJob j;
  j.fn = fn;
  j.arg = arg;
  j.chunks = chunks;
  p.run(j);
}

size_t Ctx::tbeg(const char* name, hipStream_t st) {
  last_mark = (size_t)-1;
  if (!timing) return last_mark;
  hipEvent_t ev;
  if (hipEventCreate(&ev) != hipSuccess) return last_mark;
  (void)hipEventRecord(ev, st ? st : stream);
  pending.push_back({name, ev, nullptr});
  last_mark = pending.size() - 1;
  return last_mark;
}

void Ctx::tend(size_t idx, hipStream_t st) {
  if (!timing || idx >= pending.size() || pending[idx].e1) return;
  hipEvent_t ev;
  if (hipEventCreate(&ev) != hipSuccess) return;
  (void)hipEventRecord(ev, st ? st : stream);
  pending[idx].e1 = ev;
}

std::vector<uint32_t> Ctx::cu_mask(uint32_t count, bool in) const {
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device);
  if (ncu <= 0) ncu = 256;
  std::vector<uint32_t> m((ncu + 31) / 32, 0u);
  std::vector<bool> res(ncu, false);
  // count/8 CUs per XCD.  Bit i = 32 j + (j + s (32/per)) mod 32 is balanced over the
  // 8 XCDs whether the driver maps mask bits to XCDs contiguously (i / 32) or
  // interleaved (i mod 8).
  const uint32_t per = count / 8;
  if (ncu == 256 && per)
    for (uint32_t j = 0; j < 8; ++j)
      for (uint32_t s = 0; s < per; ++s) res[32 * j + (j + (s * 32) / per) % 32] = true;
  for (int i = 0; i < ncu; ++i)
    if (res[i] == in) m[i / 32] |= 1u << (i % 32);
  return m;
}

// masked: 0 none, 3 the GA set, 4 its complement
static hipStream_t make_stream(const Ctx* c, int masked) {
  hipStream_t s = nullptr;
  if (masked) {
    std::vector<uint32_t> m = c->cu_mask(c->ga_cus, masked == 3);
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()) == hipSuccess) return s;
    s = nullptr;
  }
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) s = nullptr;
  return s;
}

hipStream_t Ctx::side_stream(int k) {
  k %= NSIDE;
  if (!side[k]) side[k] = make_stream(this, ga_cus ? (k == 0 ? 3 : 4) : 0);
  return side[k] ? side[k] : stream;
}

int Ctx::sync() {
  int rc = hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
  // fold finished event pairs; pairs of work still running on another stream
  // (a launched collect batch while the recovery stream syncs) stay pending
  std::vector<PendingEvent> keep;
  for (auto& p : pending) {
    if (p.e1 && hipEventQuery(p.e1) == hipErrorNotReady) {
      keep.push_back(p);
      continue;
    }
    if (p.e1) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, p.e0, p.e1) == hipSuccess) {
        auto& t = times[p.name];
        t.ms += ms;
        t.launches += 1;
      }
      (void)hipEventDestroy(p.e1);
    }
    (void)hipEventDestroy(p.e0);
  }
  pending.swap(keep);
  // the launch checks read hipGetLastError: the best-effort timing queries above
  // (not-ready events, pairs split over streams) must not surface as the next
  // launch's failure
  (void)hipGetLastError();
  return rc;
}

uint32_t choose_window(uint32_t ebits) {
  // minimise squarings + window multiplies + table build
  uint32_t best_w = 1;
  double best = 1e30;
  for (uint32_t w = 1; w <= 6; ++w) {
    double cost = (double)ebits + (double)((ebits + w - 1) / w) + (double)(1u << w);
    if (cost < best) {
      best = cost;
      best_w = w;
    }
  }
  return best_w;
}

// Launch one modexp job whose descriptors are already in device memory.
// Sliding-window width for an exponent of `ebits` bits: 2^(w-1) odd powers plus
// about ebits / (w + 1) window products, fewest total (2048 bits: w = 6)
uint32_t choose_slide_window(uint32_t ebits) {
  uint32_t best_w = 1;
  double best = 1e30;
  for (uint32_t w = 1; w <= 7; ++w) {
    const double cost = (double)(1u << (w - 1)) + (double)ebits / (double)(w + 1);
    if (cost < best) {
      best = cost;
      best_w = w;
    }
  }
  return best_w;
}

int launch_modexp_desc(Ctx* c, uint32_t k32, uint32_t count, uint32_t exp_bits, const uint8_t* d_desc,
                       const uint32_t* d_consts, uint32_t* d_out, hipStream_t st, const char* table_tag,
                       uint32_t prio, uint32_t group, uint32_t desc_flags, const SplitArgs* split) {
  if (!st) st = c->stream;
  if (count == 0) return FSDKR_OK;
  // sliding windows: the 4096-bit group shapes, public exponents, wave-uniform (caller)
  // a forced context setting wins (tuning, tests), except that the 32-lane shape
  // runs only where the caller asked for it (it prepared KD = 160 constants)
  uint32_t grp = c->modexp_group ? c->modexp_group : group;
  if (grp == kWideGroup && (group != kWideGroup || k32 != 128)) grp = 16;
  if (grp == kWaveGroup && k32 != 128) grp = 16;
  if (c->ct) grp = 0;   // the regular-access kernels have one shape per width
  // sliding windows: the 4096-bit 4/8/16/32-lane shapes, public exponents, waves of
  // `group` lanes uniform (caller), so only at the caller's lane count
  const bool slide = (desc_flags & kDescSlide) && (desc_flags & kDescOutIdx) && k32 == 128 && !c->ct &&
                     grp == group && (grp == 4 || grp == 8 || grp == 16 || grp == kWideGroup);
  const int KD = table_digits(k32, grp);
  if (!KD) {
    c->fail("unsupported modulus width %u limbs", k32);
    return FSDKR_E_UNSUPPORTED;
  }
  const uint32_t ebits = exp_bits ? exp_bits : 1;
  const uint32_t w = slide ? choose_slide_window(ebits) : choose_window(ebits);
  const uint32_t nwin = (ebits + w - 1) / w;
  const size_t entries = slide ? ((size_t)1 << (w - 1)) + 1 : (size_t)1 << w;
  uint32_t* d_table = (uint32_t*)c->buf(table_tag, sizeof(uint32_t) * (size_t)count * entries * KD);
  if (!d_table) {
    c->fail("device allocation failed (%u instances, window %u)", count, w);
    return FSDKR_E_OOM;
  }
  const size_t n8 = (size_t)count * 8, n4 = (size_t)count * 4;
  ModexpArgs a;
  a.base_ptr = reinterpret_cast<const uint64_t*>(d_desc);
  a.exp_ptr = reinterpret_cast<const uint64_t*>(d_desc + n8);
  a.base_len = reinterpret_cast<const uint32_t*>(d_desc + 2 * n8);
  a.exp_len = reinterpret_cast<const uint32_t*>(d_desc + 2 * n8 + n4);
  a.mod_idx = reinterpret_cast<const uint32_t*>(d_desc + 2 * n8 + 2 * n4);
  a.nwin_i = reinterpret_cast<const uint32_t*>(d_desc + 2 * n8 + 3 * n4);
  a.nwin = nwin;
  a.window = w;
  a.consts = d_consts;
  a.out = d_out;
  a.table = d_table;
  a.count = count;
  a.prio = prio;
  a.group = grp;
  a.ct = c->ct ? 1u : 0u;
  a.slide = slide ? 1u : 0u;
  a.out_idx = (desc_flags & kDescOutIdx) ? reinterpret_cast<const uint32_t*>(d_desc + 2 * n8 + 4 * n4) : nullptr;
  if (split && split->lo_bit) {   // head / tail of split chains: the slide shapes at the caller's lanes
    if (!slide || grp != group || !(grp == 4 || grp == 8 || grp == 16 || grp == kWideGroup)) {
      c->fail("split chains need the 4 / 8 / 16 / 32-lane sliding-window shapes (group %u)", grp);
      return FSDKR_E_ARG;
    }
    const std::string base(table_tag);
    a.lo_bit = split->lo_bit;
    a.tail = split->tail ? 1u : 0u;
    a.state = (uint32_t*)c->buf((base + "_state").c_str(), (size_t)count * KD * 4);
    if (!a.state) {
      c->fail("device allocation failed (split chain state)");
      return FSDKR_E_OOM;
    }
    if (split->tail && split->d_desc2) {
      a.base2_ptr = reinterpret_cast<const uint64_t*>(split->d_desc2);
      a.exp2_ptr = reinterpret_cast<const uint64_t*>(split->d_desc2 + n8);
      a.exp2_len = reinterpret_cast<const uint32_t*>(split->d_desc2 + 2 * n8);
      a.table2 = (uint32_t*)c->buf((base + "_t2").c_str(), (size_t)count * 16 * KD * 4);
      if (!a.table2) {
        c->fail("device allocation failed (joint table)");
        return FSDKR_E_OOM;
      }
    }
  }
  const size_t tm = c->tbeg("modexp", st);
  int rc = c->hip_check(modexp(k32, a, st), "modexp launch");
  c->tend(tm, st);
  return rc;
}

void ModexpJob::pack(std::vector<uint8_t>& dst) const {
  const size_t n8 = size() * 8, n4 = size() * 4;
  const size_t o = dst.size();
  dst.resize(o + desc_bytes());
  memcpy(dst.data() + o, base_ptr.data(), n8);
  memcpy(dst.data() + o + n8, exp_ptr.data(), n8);
  memcpy(dst.data() + o + 2 * n8, base_len.data(), n4);
  memcpy(dst.data() + o + 2 * n8 + n4, exp_len.data(), n4);
  memcpy(dst.data() + o + 2 * n8 + 2 * n4, mod_idx.data(), n4);
  const uint32_t w = choose_window(exp_bits ? exp_bits : 1);
  uint32_t* nw = reinterpret_cast<uint32_t*>(dst.data() + o + 2 * n8 + 3 * n4);
  for (size_t k = 0; k < size(); ++k) nw[k] = ebits[k] ? (ebits[k] + w - 1) / w : 1u;
  if (!out_idx.empty()) memcpy(dst.data() + o + 2 * n8 + 4 * n4, out_idx.data(), n4);
}

// Upload a modexp descriptor set and launch it against prepared constants.
int launch_modexp_job(Ctx* c, const ModexpJob& job, const uint32_t* d_consts, uint32_t* d_out, const char* tag,
                      uint32_t group, uint32_t desc_flags) {
  const uint32_t count = (uint32_t)job.size();
  if (count == 0) return FSDKR_OK;
  std::string dname = std::string("mxdesc_") + tag;
  uint8_t* d_desc = (uint8_t*)c->buf(dname.c_str(), job.desc_bytes());
  if (!d_desc) {
    c->fail("device allocation failed (descriptors)");
    return FSDKR_E_OOM;
  }
  std::vector<uint8_t>& h = c->staging;
  h.clear();
  job.pack(h);
  int rc = c->hip_check(hipMemcpyAsync(d_desc, h.data(), h.size(), hipMemcpyHostToDevice, c->stream), "H2D modexp desc");
  if (rc) return rc;
  // the staging buffer is reused by the next call: make this copy complete first
  rc = c->hip_check(hipStreamSynchronize(c->stream), "sync desc");
  if (rc) return rc;
  return launch_modexp_desc(c, job.k32, count, job.exp_bits, d_desc, d_consts, d_out, nullptr, "mxtable", c->prio,
                            group, desc_flags);
}

int setup_moduli(Ctx* c, uint32_t k32, const uint32_t* d_mods, uint32_t n_mod, uint32_t** d_consts, const char* tag,
                 uint32_t group, bool wave) {
  const int KD = shape_digits_g(k32, group);
  if (!KD) {
    c->fail("unsupported modulus width %u limbs", k32);
    return FSDKR_E_UNSUPPORTED;
  }
  std::string name = std::string("consts_") + tag;
  *d_consts = (uint32_t*)c->buf(name.c_str(), sizeof(uint32_t) * (size_t)cons_stride(KD) * (n_mod ? n_mod : 1));
  if (!*d_consts) {
    c->fail("device allocation failed (mod consts)");
    return FSDKR_E_OOM;
  }
  c->mark("mod_setup", true);
  int rc = c->hip_check(wave && !group ? mod_setup_wave(k32, d_mods, n_mod, *d_consts, c->stream)
                                       : mod_setup_g(k32, group, d_mods, n_mod, *d_consts, c->stream),
                        "mod_setup launch");
  c->mark("mod_setup", false);
  return rc;
}

// Runs mod_setup + modexp on device-resident contiguous operands.
int run_modexp_device(Ctx* c, uint32_t k32, uint32_t count, const uint32_t* d_base, const uint32_t* d_exp,
                      uint32_t exp_limbs, uint32_t exp_bits, const uint32_t* d_mod_idx, const uint32_t* d_mods,
                      uint32_t n_mod, uint32_t* d_out) {
  if (count == 0) return FSDKR_OK;
  uint32_t* d_consts = nullptr;
  // a context forced to the 32-lane shape (tuning, tests) gets KD = 160 constants here
  const uint32_t wide = (!c->ct && c->modexp_group == kWideGroup && k32 == 128) ? kWideGroup : 0u;
  int rc = setup_moduli(c, k32, d_mods, n_mod, &d_consts, wide ? "generic_wide" : "generic", wide);
  if (rc) return rc;
  ModexpJob job;
  job.k32 = k32;
  job.exp_bits = exp_bits;
  job.base_ptr.resize(count);
  job.exp_ptr.resize(count);
  job.base_len.assign(count, k32);
  job.exp_len.assign(count, exp_limbs);
  job.ebits.assign(count, exp_bits);
  job.mod_idx.resize(count);
  for (uint32_t i = 0; i < count; ++i) {
    job.base_ptr[i] = (uint64_t)(uintptr_t)(d_base + (size_t)i * k32);
    job.exp_ptr[i] = (uint64_t)(uintptr_t)(d_exp + (size_t)i * exp_limbs);
  }
  rc = c->hip_check(hipMemcpyAsync(job.mod_idx.data(), d_mod_idx, sizeof(uint32_t) * count, hipMemcpyDeviceToHost,
                                   c->stream),
                    "D2H mod_idx");
  if (rc) return rc;
  rc = c->hip_check(hipStreamSynchronize(c->stream), "sync");
  if (rc) return rc;
  return launch_modexp_job(c, job, d_consts, d_out, "generic", wide);
}

// Exponent per modulus (key): d_exp is [n_mod][exp_limbs].  The instances are
// regrouped by key so the instances of every wave share their exponent (runs
// padded to whole waves with copies that rewrite their own row), which lets the
// 4096-bit shapes run sliding windows (modexp_slide_kernel: 2048-bit exponent at
// w = 6, ~2042 squarings + ~300 products against 2043 + 440 with fixed 5-bit
// windows).  Other widths, or a constant-time context, keep fixed windows.
int run_modexp_keyed(Ctx* c, uint32_t k32, uint32_t count, const uint32_t* d_base, const uint32_t* d_exp,
                     uint32_t exp_limbs, uint32_t exp_bits, const uint32_t* d_mod_idx, const uint32_t* d_mods,
                     uint32_t n_mod, uint32_t* d_out) {
  if (count == 0) return FSDKR_OK;
  uint32_t* d_consts = nullptr;
  int rc = setup_moduli(c, k32, d_mods, n_mod, &d_consts, "keyed", 0);
  if (rc) return rc;
  std::vector<uint32_t> idx(count);
  rc = c->hip_check(hipMemcpyAsync(idx.data(), d_mod_idx, sizeof(uint32_t) * count, hipMemcpyDeviceToHost, c->stream),
                    "D2H mod_idx");
  if (rc) return rc;
  if ((rc = c->hip_check(hipStreamSynchronize(c->stream), "sync"))) return rc;
  ModexpJob job;
  job.k32 = k32;
  for (uint32_t i = 0; i < count; ++i) {
    if (idx[i] >= n_mod) {
      c->fail("fsdkr_modexp_keyed_device: mod_idx[%u] = %u out of range (%u moduli)", i, idx[i], n_mod);
      return FSDKR_E_ARG;
    }
    job.add((uint64_t)(uintptr_t)(d_base + (size_t)i * k32), k32, (uint64_t)(uintptr_t)(d_exp + (size_t)idx[i] * exp_limbs),
            exp_limbs, exp_bits, idx[i]);
  }
  job.exp_bits = exp_bits;
  const uint32_t G = keyed_lanes(count);
  uint32_t flags = 0;   // the regrouped job carries out_idx (the caller's rows)
  if (k32 == 128 && !c->ct && group_by_exponent(job, 64 / G, kPadSelf)) flags = kDescOutIdx | kDescSlide;
  return launch_modexp_job(c, job, d_consts, d_out, "keyed", (flags & kDescSlide) ? G : 0u, flags);
}

}  // namespace fsdkr

// ---------------------------------------------------------------- C ABI -------
extern "C" {

int fsdkr_device_available(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n > 0 ? 1 : 0;
}

int fsdkr_ctx_create(const fsdkr_cfg* cfg, fsdkr_ctx** out) {
  if (!out) return FSDKR_E_ARG;
  *out = nullptr;
  Ctx* c = new (std::nothrow) Ctx();
  if (!c) return FSDKR_E_OOM;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    delete c;
    return FSDKR_E_HIP;
  }
  int dev = cfg ? cfg->device : -1;
  if (dev >= 0) {
    if (dev >= n || hipSetDevice(dev) != hipSuccess) {
      delete c;
      return FSDKR_E_ARG;
    }
  } else {
    (void)hipGetDevice(&dev);
  }
  c->device = dev;
  c->flags = cfg ? cfg->flags : 0u;
  c->timing = (c->flags & FSDKR_CFG_TIMING) != 0;
  if (!(c->stream = make_stream(c, 0))) {
    delete c;
    return FSDKR_E_HIP;
  }
  *out = reinterpret_cast<fsdkr_ctx*>(c);
  return FSDKR_OK;
}

void fsdkr_ctx_destroy(fsdkr_ctx* ctx) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return;
  (void)c->sync();
  for (auto& kv : c->bufs)
    if (kv.second.ptr) (void)hipFree(kv.second.ptr);
  for (auto& sd : c->side)
    if (sd) (void)hipStreamDestroy(sd);
  if (c->aux) (void)hipStreamDestroy(c->aux);
  if (c->pinned) (void)hipHostFree(c->pinned);
  for (auto& kv : c->hbufs)
    if (kv.second.ptr) (void)hipHostFree(kv.second.ptr);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  fsdkr::free_collect_plan(c);
  fsdkr::free_ga_pre(c);
  fsdkr::free_recover(c);
  if (c->span_beg) (void)hipEventDestroy(c->span_beg);
  if (c->span_end) (void)hipEventDestroy(c->span_end);
  delete c;
}

int Ctx::span_begin(hipStream_t st) {
  if (!span_beg && hipEventCreate(&span_beg) != hipSuccess) return hip_check(hipErrorOutOfMemory, "span event");
  if (!span_end && hipEventCreate(&span_end) != hipSuccess) return hip_check(hipErrorOutOfMemory, "span event");
  span_armed = true;
  span_ms = -1.0f;
  return hip_check(hipEventRecord(span_beg, st), "span event record");
}

uint32_t fsdkr_collect_reuse_mask(const fsdkr_ctx* ctx) {
  const Ctx* c = reinterpret_cast<const Ctx*>(ctx);
  return c ? c->reuse_mask : 0u;
}

double fsdkr_collect_last_span_ms(const fsdkr_ctx* ctx) {
  const Ctx* c = reinterpret_cast<const Ctx*>(ctx);
  return c ? (double)c->span_ms : -1.0;
}

const char* fsdkr_last_error(const fsdkr_ctx* ctx) {
  const Ctx* c = reinterpret_cast<const Ctx*>(ctx);
  return c ? c->err.c_str() : "null context";
}

int fsdkr_ctx_set_modexp_group(fsdkr_ctx* ctx, uint32_t lanes) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c || (lanes != 0 && lanes != 2 && lanes != 4 && lanes != 8 && lanes != 16 && lanes != 32 && lanes != 64)) return FSDKR_E_ARG;
  c->modexp_group = lanes;
  return FSDKR_OK;
}

int fsdkr_ctx_set_cu_split(fsdkr_ctx* ctx, uint32_t ga_cus) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c || (ga_cus && (ga_cus % 8 != 0 || ga_cus > 224))) return FSDKR_E_ARG;
  if (c->ga_cus == ga_cus) return FSDKR_OK;
  int rc = c->sync();
  if (rc) return rc;
  // every stream is re-created lazily with the new masks
  if ((rc = c->hip_check(hipDeviceSynchronize(), "sync"))) return rc;
  for (auto& sd : c->side)
    if (sd) {
      (void)hipStreamDestroy(sd);
      sd = nullptr;
    }
  if (c->aux) (void)hipStreamDestroy(c->aux);
  c->aux = nullptr;
  c->ga_cus = ga_cus;
  hipStream_t s = make_stream(c, ga_cus ? 4 : 0);
  if (!s) return FSDKR_E_HIP;
  (void)hipStreamDestroy(c->stream);
  c->stream = s;
  return FSDKR_OK;
}

int fsdkr_ctx_set_timing(fsdkr_ctx* ctx, int on) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  int rc = c->sync();   // fold events of launches made under the old setting
  c->timing = on != 0;
  c->flags = on ? (c->flags | FSDKR_CFG_TIMING) : (c->flags & ~FSDKR_CFG_TIMING);
  return rc;
}

int fsdkr_ctx_set_flags(fsdkr_ctx* ctx, uint32_t flags) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  int rc = c->sync();
  c->flags = flags;
  c->timing = (flags & FSDKR_CFG_TIMING) != 0;
  return rc;
}

int fsdkr_mod_inverse(fsdkr_ctx* ctx, uint32_t mod_limbs, uint32_t count, const uint32_t* y, const uint32_t* m,
                      uint32_t* out, uint32_t* unit) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  if (count == 0) return FSDKR_OK;
  if (!y || !m || !unit) {
    c->fail("fsdkr_mod_inverse: null pointer");
    return FSDKR_E_ARG;
  }
  if (!shape_digits(mod_limbs)) {
    c->fail("fsdkr_mod_inverse: unsupported modulus width %u limbs", mod_limbs);
    return FSDKR_E_UNSUPPORTED;
  }
  for (uint32_t i = 0; i < count; ++i)
    if ((m[(size_t)i * mod_limbs] & 1u) == 0) {
      c->fail("fsdkr_mod_inverse: modulus %u is even", i);
      return FSDKR_E_ARG;
    }
  const size_t nb = sizeof(uint32_t) * (size_t)count * mod_limbs;
  uint8_t* d = (uint8_t*)c->buf("inv_io", 3 * nb + 2 * 8 * (size_t)count + 4 * (size_t)count + 1024);
  if (!d) {
    c->fail("fsdkr_mod_inverse: device allocation failed");
    return FSDKR_E_OOM;
  }
  uint32_t* d_y = (uint32_t*)d;
  uint32_t* d_m = (uint32_t*)(d + nb);
  uint32_t* d_o = (uint32_t*)(d + 2 * nb);
  uint64_t* d_yp = (uint64_t*)(d + 3 * nb);
  uint64_t* d_mp = d_yp + count;
  uint32_t* d_u = (uint32_t*)(d_mp + count);
  std::vector<uint64_t> ptrs(2 * (size_t)count);
  for (uint32_t i = 0; i < count; ++i) {
    ptrs[i] = (uint64_t)(uintptr_t)(d_y + (size_t)i * mod_limbs);
    ptrs[count + i] = (uint64_t)(uintptr_t)(d_m + (size_t)i * mod_limbs);
  }
  int rc;
  if ((rc = c->hip_check(hipMemcpyAsync(d_y, y, nb, hipMemcpyHostToDevice, c->stream), "H2D y")) ||
      (rc = c->hip_check(hipMemcpyAsync(d_m, m, nb, hipMemcpyHostToDevice, c->stream), "H2D m")) ||
      (rc = c->hip_check(hipMemcpyAsync(d_yp, ptrs.data(), ptrs.size() * 8, hipMemcpyHostToDevice, c->stream),
                         "H2D ptrs")))
    return rc;
  // instances sharing a modulus (equal rows) are inverted together (Montgomery's
  // simultaneous inversion, inverse_batch_kernel) where the width has that shape
  std::vector<uint32_t> order(count), gstart;
  for (uint32_t i = 0; i < count; ++i) order[i] = i;
  const size_t kd = batch_inv_on(c) ? inverse_batch_scratch_words(mod_limbs) : 0;
  if (kd) {
    auto row = [&](uint32_t i) { return m + (size_t)i * mod_limbs; };
    std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y2) {
      return memcmp(row(x), row(y2), 4 * (size_t)mod_limbs) < 0;
    });
    for (uint32_t t = 0; t < count; ++t)
      if (t == 0 || memcmp(row(order[t]), row(order[t - 1]), 4 * (size_t)mod_limbs) != 0) gstart.push_back(t);
    gstart.push_back(count);
  }
  c->mark("inverse", true);
  if (kd && gstart.size() - 1 < count) {
    uint8_t* g = (uint8_t*)c->buf("inv_grp", 4 * ((size_t)count + gstart.size()) + 1024);
    uint32_t* scr = (uint32_t*)c->buf("inv_grp_scratch", (size_t)count * kd * 4);
    if (!g || !scr) {
      c->fail("fsdkr_mod_inverse: device allocation failed");
      return FSDKR_E_OOM;
    }
    uint32_t* d_ord = (uint32_t*)g;
    uint32_t* d_gs = d_ord + count;
    if ((rc = c->hip_check(hipMemcpyAsync(d_ord, order.data(), 4 * (size_t)count, hipMemcpyHostToDevice, c->stream),
                           "H2D order")) ||
        (rc = c->hip_check(hipMemcpyAsync(d_gs, gstart.data(), 4 * gstart.size(), hipMemcpyHostToDevice, c->stream),
                           "H2D groups")))
      return rc;
    BatchInverseArgs b{d_yp, d_mp, d_ord, d_gs, d_o, d_u, scr, (uint32_t)gstart.size() - 1};
    rc = c->hip_check(launch_inverse_batch(mod_limbs, b, c->stream), "batch inverse launch");
    if (!rc) rc = c->sync();   // (the host order / group vectors go out of scope)
  } else {
    InverseArgs a{d_yp, d_mp, d_o, d_u, nullptr, count};
    rc = c->hip_check(launch_inverse(mod_limbs, a, c->stream), "inverse launch");
  }
  c->mark("inverse", false);
  if (rc) return rc;
  if (out && (rc = c->hip_check(hipMemcpyAsync(out, d_o, nb, hipMemcpyDeviceToHost, c->stream), "D2H inv")))
    return rc;
  if ((rc = c->hip_check(hipMemcpyAsync(unit, d_u, 4 * (size_t)count, hipMemcpyDeviceToHost, c->stream), "D2H unit")))
    return rc;
  return c->sync();
}

int fsdkr_modexp_batch(fsdkr_ctx* ctx, uint32_t mod_limbs, uint32_t count, const uint32_t* base,
                       const uint32_t* exp, uint32_t exp_limbs, const uint32_t* mod_idx, const uint32_t* mods,
                       uint32_t n_mod, uint32_t* out) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  if (count == 0) return FSDKR_OK;
  if (!base || !exp || !mod_idx || !mods || !out || n_mod == 0 || exp_limbs == 0) {
    c->fail("fsdkr_modexp_batch: null pointer or empty table");
    return FSDKR_E_ARG;
  }
  if (!shape_digits_g(mod_limbs, 0)) {   // the verifier's classes and 1024-bit key-generation moduli
    c->fail("fsdkr_modexp_batch: unsupported modulus width %u limbs", mod_limbs);
    return FSDKR_E_UNSUPPORTED;
  }
  for (uint32_t m = 0; m < n_mod; ++m) {
    if ((mods[(size_t)m * mod_limbs] & 1u) == 0) {
      c->fail("fsdkr_modexp_batch: modulus %u is even", m);
      return FSDKR_E_ARG;
    }
  }
  uint32_t exp_bits = 0;
  for (uint32_t i = 0; i < count; ++i) {
    if (mod_idx[i] >= n_mod) {
      c->fail("fsdkr_modexp_batch: mod_idx[%u]=%u out of range", i, mod_idx[i]);
      return FSDKR_E_ARG;
    }
    const uint32_t* e = exp + (size_t)i * exp_limbs;
    for (int k = (int)exp_limbs - 1; k >= 0; --k) {
      if (e[k]) {
        uint32_t b = 32u * (uint32_t)k + 32u - (uint32_t)__builtin_clz(e[k]);
        if (b > exp_bits) exp_bits = b;
        break;
      }
    }
  }
  const size_t nb = sizeof(uint32_t) * (size_t)count * mod_limbs;
  const size_t ne = sizeof(uint32_t) * (size_t)count * exp_limbs;
  uint32_t* d_base = (uint32_t*)c->buf("mx_base", nb);
  uint32_t* d_exp = (uint32_t*)c->buf("mx_exp", ne);
  uint32_t* d_idx = (uint32_t*)c->buf("mx_idx", sizeof(uint32_t) * count);
  uint32_t* d_mods = (uint32_t*)c->buf("mx_mods", sizeof(uint32_t) * (size_t)n_mod * mod_limbs);
  uint32_t* d_out = (uint32_t*)c->buf("mx_out", nb);
  if (!d_base || !d_exp || !d_idx || !d_mods || !d_out) {
    c->fail("fsdkr_modexp_batch: device allocation failed");
    return FSDKR_E_OOM;
  }
  int rc;
  if ((rc = c->hip_check(hipMemcpyAsync(d_base, base, nb, hipMemcpyHostToDevice, c->stream), "H2D base"))) return rc;
  if ((rc = c->hip_check(hipMemcpyAsync(d_exp, exp, ne, hipMemcpyHostToDevice, c->stream), "H2D exp"))) return rc;
  if ((rc = c->hip_check(hipMemcpyAsync(d_idx, mod_idx, sizeof(uint32_t) * count, hipMemcpyHostToDevice, c->stream),
                         "H2D idx")))
    return rc;
  if ((rc = c->hip_check(hipMemcpyAsync(d_mods, mods, sizeof(uint32_t) * (size_t)n_mod * mod_limbs,
                                        hipMemcpyHostToDevice, c->stream),
                         "H2D mods")))
    return rc;
  rc = run_modexp_device(c, mod_limbs, count, d_base, d_exp, exp_limbs, exp_bits, d_idx, d_mods, n_mod, d_out);
  if (rc) return rc;
  if ((rc = c->hip_check(hipMemcpyAsync(out, d_out, nb, hipMemcpyDeviceToHost, c->stream), "D2H out"))) return rc;
  return c->sync();
}

int fsdkr_modexp_batch_ct(fsdkr_ctx* ctx, uint32_t mod_limbs, uint32_t count, const uint32_t* base,
                          const uint32_t* exp, uint32_t exp_limbs, const uint32_t* mod_idx, const uint32_t* mods,
                          uint32_t n_mod, uint32_t* out) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  CtScope ct(c);
  return fsdkr_modexp_batch(ctx, mod_limbs, count, base, exp, exp_limbs, mod_idx, mods, n_mod, out);
}

int fsdkr_modexp_batch_device(fsdkr_ctx* ctx, uint32_t mod_limbs, uint32_t count, const uint32_t* d_base,
                              const uint32_t* d_exp, uint32_t exp_limbs, uint32_t exp_bits,
                              const uint32_t* d_mod_idx, const uint32_t* d_mods, uint32_t n_mod, uint32_t* d_out) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  if (count == 0) return FSDKR_OK;
  if (!d_base || !d_exp || !d_mod_idx || !d_mods || !d_out || n_mod == 0 || exp_limbs == 0 ||
      exp_bits > 32u * exp_limbs) {
    c->fail("fsdkr_modexp_batch_device: bad argument");
    return FSDKR_E_ARG;
  }
  int rc = run_modexp_device(c, mod_limbs, count, d_base, d_exp, exp_limbs, exp_bits, d_mod_idx, d_mods, n_mod, d_out);
  if (rc) return rc;
  return c->sync();
}

int fsdkr_modexp_keyed_device(fsdkr_ctx* ctx, uint32_t mod_limbs, uint32_t count, const uint32_t* d_base,
                              const uint32_t* d_exp, uint32_t exp_limbs, uint32_t exp_bits,
                              const uint32_t* d_mod_idx, const uint32_t* d_mods, uint32_t n_mod, uint32_t* d_out) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  if (count == 0) return FSDKR_OK;
  if (!d_base || !d_exp || !d_mod_idx || !d_mods || !d_out || n_mod == 0 || exp_limbs == 0 ||
      exp_bits > 32u * exp_limbs) {
    c->fail("fsdkr_modexp_keyed_device: bad argument");
    return FSDKR_E_ARG;
  }
  int rc = run_modexp_keyed(c, mod_limbs, count, d_base, d_exp, exp_limbs, exp_bits, d_mod_idx, d_mods, n_mod, d_out);
  if (rc) return rc;
  return c->sync();
}

int fsdkr_kernel_time(const fsdkr_ctx* ctx, const char* name, double* ms, uint32_t* launches) {
  const Ctx* c = reinterpret_cast<const Ctx*>(ctx);
  if (!c || !name) return FSDKR_E_ARG;
  auto it = c->times.find(name);
  if (ms) *ms = (it == c->times.end()) ? 0.0 : it->second.ms;
  if (launches) *launches = (it == c->times.end()) ? 0u : it->second.launches;
  return FSDKR_OK;
}

void fsdkr_kernel_time_reset(fsdkr_ctx* ctx) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (c) c->times.clear();
}

}  // extern "C"
