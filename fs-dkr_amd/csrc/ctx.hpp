// Internal context object behind the opaque fsdkr_ctx handle.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <map>
#include <string>
#include <unordered_map>
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
  uint32_t flags = 0;   // fsdkr_cfg flags (FSDKR_CFG_*)
  std::string err;
  std::map<std::string, DevBuf> bufs;
  std::map<std::string, TimeAcc> times;
  std::vector<PendingEvent> pending;
  std::vector<uint8_t> staging;   // host staging for descriptor uploads
  static constexpr int NSIDE = 11;
  hipStream_t side[NSIDE] = {};   // concurrent streams for independent jobs (lazily created)
  void* plan = nullptr;           // prepared collect() batch (collect.cpp)
  void* ga_pre = nullptr;         // prestarted s^N mod N^2 job (fsdkr_collect_prestart)
  void* recover = nullptr;        // launched share recovery (fsdkr_collect_recover_launch)
  // pinned host arena for the collect() image (grow-only; one H2D copy per prepare)
  uint8_t* pinned = nullptr;
  size_t pinned_bytes = 0;
  uint8_t* host_arena(size_t bytes);
  // named grow-only pinned host buffers (a prestart's image, kept for prepare's match)
  std::map<std::string, DevBuf> hbufs;
  uint8_t* host_buf(const char* name, size_t bytes);
  // stream of the share-recovery entry points (decrypt, MSM): separate from the
  // collect pipeline so they overlap a launched batch (fsdkr_collect_launch)
  hipStream_t aux = nullptr;
  hipStream_t aux_stream();

  void fail(const char* fmt, ...);
  int hip_check(hipError_t e, const char* what);
  // grow-only named device buffer (contents undefined after growth)
  void* buf(const char* name, size_t bytes);
  // HIP-event brackets around a kernel launch (timing mode only); st = nullptr: main stream
  void mark(const char* name, bool begin, hipStream_t st = nullptr) {
    if (begin) tbeg(name, st ? st : stream); else tend(last_mark, st ? st : stream);
  }
  size_t tbeg(const char* name, hipStream_t st);
  void tend(size_t idx, hipStream_t st);
  size_t last_mark = (size_t)-1;
  uint32_t modexp_group = 0;   // lanes per modexp instance (0 = by batch size)
  // issue priority (s_setprio) of the generic entry points' kernels: the share
  // recovery raises it while it overlaps a launched collect pipeline
  uint32_t prio = 0;
  // regular-access modexp (secret exponents: prover, key generation, decryption)
  bool ct = false;
  hipStream_t side_stream(int k);
  // GA split (fsdkr_ctx_set_cu_split(G), G a multiple of 8): side stream 0 (GA,
  // the s^N mod N^2 chains) runs on G CUs spread over the XCDs, every other
  // stream (main, side, recovery) on the complement, so the longest dependent
  // chains of a small (sharded) batch never share a SIMD with the throughput jobs.
  uint32_t ga_cus = 0;
  // CU mask words of a balanced set of `count` CUs (in = true) or of its complement
  std::vector<uint32_t> cu_mask(uint32_t count, bool in) const;
  // device span of the last collect() call: a timing event at the first device
  // work of the call (prestart H2D done, else the pipeline launch) and one after
  // the pipeline's last kernel; finish turns them into span_ms
  hipEvent_t span_beg = nullptr, span_end = nullptr;
  bool span_armed = false;
  float span_ms = -1.0f;
  uint32_t reuse_mask = 0;   // prestarted parts the last prepare reused (fsdkr_collect_reuse_mask)
  int span_begin(hipStream_t st);
  // synchronise the stream and fold pending events into `times`
  int sync();
};

// Runs the calls of one C-ABI entry point on another stream (the context is
// single-threaded per the ABI, so swapping the main stream is safe).
struct StreamScope {
  Ctx* c;
  hipStream_t saved;
  StreamScope(Ctx* cx, hipStream_t s) : c(cx), saved(cx->stream) {
    if (s) c->stream = s;
  }
  ~StreamScope() { c->stream = saved; }
};

// Raises the context's kernel issue priority for the calls of one entry point.
struct PrioScope {
  Ctx* c;
  uint32_t saved;
  PrioScope(Ctx* cx, uint32_t p) : c(cx), saved(cx->prio) { c->prio = p; }
  ~PrioScope() { c->prio = saved; }
};

// Runs the modexp launches of one entry point in regular-access mode (ModexpArgs.ct).
struct CtScope {
  Ctx* c;
  bool saved;
  explicit CtScope(Ctx* cx, bool on = true) : c(cx), saved(cx->ct) { c->ct = on; }
  ~CtScope() { c->ct = saved; }
};

// Host worker threads for the collect() pre-pass (FSDKR_HOST_THREADS, else
// OMP_NUM_THREADS, else min(hardware threads, 16)).
unsigned host_threads();

// fn(arg, c) for every c in [0, chunks), on a process-wide pool of
// host_threads() - 1 parked worker threads and the calling thread; returns when
// every chunk is done.  A call from a pool worker, or while another thread's
// call runs, uses fresh threads instead (the collect() pre-pass issues a dozen
// of these per call: spawning 15 threads each time cost ~0.2-0.5 ms apiece).
void host_pool_run(size_t chunks, void (*fn)(void*, size_t), void* arg);

// A batch of modexp instances of one modulus width (k32 limbs) and one
// exponent-length class (exp_bits = max bits; sets the window count).
struct ModexpJob {
  uint32_t k32 = 0;
  uint32_t exp_bits = 0;
  std::vector<uint64_t> base_ptr, exp_ptr;   // device addresses
  std::vector<uint32_t> base_len, exp_len;   // limbs
  std::vector<uint32_t> mod_idx;
  std::vector<uint32_t> ebits;               // per-instance exponent bit bound
  // output row of each instance (empty: row = instance); a job laid out so the
  // instances of every wave share their exponent (GA receiver-major) carries it
  // and launches with sliding windows (launch_modexp_desc slide)
  std::vector<uint32_t> out_idx;
  void add(uint64_t b, uint32_t blen, uint64_t e, uint32_t elen, uint32_t eb, uint32_t m) {
    base_ptr.push_back(b);
    base_len.push_back(blen);
    exp_ptr.push_back(e);
    exp_len.push_back(elen);
    mod_idx.push_back(m);
    ebits.push_back(eb);
    if (eb > exp_bits) exp_bits = eb;
    // a job that carries output rows (group_by_exponent, append) keeps one per
    // instance: the added instance writes the next row
    if (!out_idx.empty()) out_idx.push_back((uint32_t)(size() - 1));
  }
  // append another job's instances (same modulus width): one merged launch
  void append(const ModexpJob& o) {
    const size_t base = size();
    if (!out_idx.empty() || !o.out_idx.empty()) {   // rows of the appended part follow this job's rows
      for (size_t k = out_idx.size(); k < base; ++k) out_idx.push_back((uint32_t)k);
      for (size_t k = 0; k < o.size(); ++k) out_idx.push_back((uint32_t)(base + (o.out_idx.empty() ? k : o.out_idx[k])));
    }
    base_ptr.insert(base_ptr.end(), o.base_ptr.begin(), o.base_ptr.end());
    exp_ptr.insert(exp_ptr.end(), o.exp_ptr.begin(), o.exp_ptr.end());
    base_len.insert(base_len.end(), o.base_len.begin(), o.base_len.end());
    exp_len.insert(exp_len.end(), o.exp_len.begin(), o.exp_len.end());
    mod_idx.insert(mod_idx.end(), o.mod_idx.begin(), o.mod_idx.end());
    ebits.insert(ebits.end(), o.ebits.begin(), o.ebits.end());
    if (o.exp_bits > exp_bits) exp_bits = o.exp_bits;
  }
  size_t size() const { return base_ptr.size(); }
  size_t desc_bytes() const { return size() * (8 + 8 + 4 + 4 + 4 + 4 + (out_idx.empty() ? 0 : 4)); }
  // append base_ptr | exp_ptr | base_len | exp_len | mod_idx | nwin (window of choose_window(exp_bits))
  // [| out_idx]
  void pack(std::vector<uint8_t>& dst) const;
};

uint32_t choose_window(uint32_t ebits);
// launch_modexp_desc desc_flags: the descriptors end with out_idx (ModexpJob.out_idx);
// the instances of every wave share their exponent (sliding windows)
constexpr uint32_t kDescOutIdx = 1, kDescSlide = 2;

// J1 (s2^N_i | s^N_i mod N_i^2) regrouped so the instances of every wave share
// their exponent N_i: stable order by exponent address (receiver), out_idx = the
// original row.  With a scratch output row (pad_row != kNoPad) every run of one
// exponent is padded to whole waves of `per_wave` instances with copies of its
// last chain writing pad_row (at most per_wave - 1 per receiver); returns whether
// every wave is then uniform (the launch may use sliding windows: kDescSlide).
// pad_row == kPadSelf: a pad copy writes its chain's own row (the same value
// twice, no scratch row needed)
constexpr uint32_t kNoPad = 0xffffffffu, kPadSelf = 0xfffffffeu;
// lanes per instance of a keyed 4096-bit launch, as the generic launch picks them
// (modexp.hip pick_group): the widest shape whose lanes fit the resident-wave capacity
inline uint32_t keyed_lanes(size_t count) {
  constexpr uint64_t kLaneCapacity = 256ull * 4 * 3 * 64;
  return (uint64_t)count * 16 <= kLaneCapacity ? 16u : (uint64_t)count * 8 <= kLaneCapacity ? 8u : 4u;
}
inline bool group_by_exponent(ModexpJob& J, uint32_t per_wave, uint32_t pad_row) {
  const size_t cnt = J.size();
  // stable order by exponent address: a counting sort over the few distinct
  // addresses (a comparison sort of 131k instances cost ~10 ms at n = 256).  The
  // distinct addresses are found by hashing (first-seen ids), then only they are
  // sorted: O(instances) on the path before GA's launch
  std::unordered_map<uint64_t, uint32_t> seen;
  seen.reserve(512);
  std::vector<uint64_t> keys;
  std::vector<uint32_t> kid(cnt), ord(cnt);
  for (size_t k = 0; k < cnt; ++k) {
    const auto it = seen.emplace(J.exp_ptr[k], (uint32_t)keys.size());
    if (it.second) keys.push_back(J.exp_ptr[k]);
    kid[k] = it.first->second;
  }
  std::vector<uint32_t> rank(keys.size());
  {
    std::vector<uint32_t> by(keys.size());
    for (uint32_t q = 0; q < (uint32_t)by.size(); ++q) by[q] = q;
    std::sort(by.begin(), by.end(), [&](uint32_t x, uint32_t y) { return keys[x] < keys[y]; });
    for (uint32_t q = 0; q < (uint32_t)by.size(); ++q) rank[by[q]] = q;
  }
  std::vector<uint32_t> start(keys.size() + 1, 0);
  for (size_t k = 0; k < cnt; ++k) {
    kid[k] = rank[kid[k]];
    ++start[kid[k] + 1];
  }
  for (size_t q = 1; q < start.size(); ++q) start[q] += start[q - 1];
  for (size_t k = 0; k < cnt; ++k) ord[start[kid[k]]++] = (uint32_t)k;
  auto same = [&](uint32_t x, uint32_t y) {
    return J.exp_ptr[x] == J.exp_ptr[y] && J.exp_len[x] == J.exp_len[y] && J.ebits[x] == J.ebits[y];
  };
  bool aligned = per_wave > 0;
  for (size_t s = 0; s < cnt && aligned && pad_row == kNoPad;) {   // unpadded: every run whole waves
    size_t e = s;
    while (e < cnt && same(ord[e], ord[s])) ++e;
    aligned = (e - s) % per_wave == 0;
    s = e;
  }
  ModexpJob G;
  G.k32 = J.k32;
  for (auto* v : {&G.base_len, &G.exp_len, &G.mod_idx, &G.ebits, &G.out_idx}) v->reserve(cnt + cnt / 8);
  G.base_ptr.reserve(cnt + cnt / 8);
  G.exp_ptr.reserve(cnt + cnt / 8);
  auto put = [&](uint32_t k, uint32_t row) {
    G.add(J.base_ptr[k], J.base_len[k], J.exp_ptr[k], J.exp_len[k], J.ebits[k], J.mod_idx[k]);
    if (G.out_idx.size() == G.size()) G.out_idx.back() = row;   // add() extended a non-empty out_idx
    else G.out_idx.push_back(row);
  };
  for (size_t s = 0; s < cnt;) {
    size_t e = s;
    while (e < cnt && same(ord[e], ord[s])) ++e;
    for (size_t q = s; q < e; ++q) put(ord[q], J.out_idx.empty() ? ord[q] : J.out_idx[ord[q]]);
    if (aligned && pad_row != kNoPad)
      for (size_t q = e - s; q % per_wave; ++q)
        put(ord[e - 1], pad_row != kPadSelf ? pad_row : J.out_idx.empty() ? ord[e - 1] : J.out_idx[ord[e - 1]]);
    s = e;
  }
  G.exp_bits = J.exp_bits;
  J = std::move(G);
  return aligned;
}
// RingPedersenProof::verify outcome from the per-index equalities and the
// challenge-length word of ped_hash (ring_pedersen_proof.rs:136-153): checks run
// in index order, so a failing check before the BitVec index panic is an error,
// not a panic.  bit0 = ok, bit1 = the reference panics.
inline uint8_t ped_verdict(const uint32_t* eq, uint32_t M, uint32_t panic_word) {
  const uint32_t readable = panic_word ? panic_word - 1 : M;
  for (uint32_t k = 0; k < readable && k < M; ++k)
    if (!eq[k]) return 0;
  return panic_word ? 2 : 1;
}
void free_collect_plan(Ctx* c);
void free_recover(Ctx* c);
void free_ga_pre(Ctx* c);
int launch_modexp_job(Ctx* c, const ModexpJob& job, const uint32_t* d_consts, uint32_t* d_out, const char* tag,
                      uint32_t group = 0, uint32_t desc_flags = 0);
// A split sliding-window launch (ModexpArgs lo_bit / tail, modexp.hip): the head
// runs the exponent bits >= lo_bit, the tail (same descriptors, group and
// table_tag) the rest, jointly with base2^exp2 when d_desc2 (per instance:
// base2_ptr u64 | exp2_ptr u64 | exp2_len u32) is set.
struct SplitArgs {
  uint32_t lo_bit = 0;
  bool tail = false;
  const uint8_t* d_desc2 = nullptr;
};
int launch_modexp_desc(Ctx* c, uint32_t k32, uint32_t count, uint32_t exp_bits, const uint8_t* d_desc,
                       const uint32_t* d_consts, uint32_t* d_out, hipStream_t st = nullptr,
                       const char* table_tag = "mxtable", uint32_t prio = 0, uint32_t group = 0,
                       uint32_t desc_flags = 0, const SplitArgs* split = nullptr);
// group: kWideGroup prepares the KD = 160 constants of the 32-lane 4096-bit shape;
// wave: the same constants from one wave per modulus where the width has that shape
// (mod_setup_wave: few VGPRs, so it is dispatched beside long-running waves)
int setup_moduli(Ctx* c, uint32_t k32, const uint32_t* d_mods, uint32_t n_mod, uint32_t** d_consts, const char* tag,
                 uint32_t group = 0, bool wave = false);
int run_modexp_device(Ctx* c, uint32_t k32, uint32_t count, const uint32_t* d_base, const uint32_t* d_exp,
                      uint32_t exp_limbs, uint32_t exp_bits, const uint32_t* d_mod_idx, const uint32_t* d_mods,
                      uint32_t n_mod, uint32_t* d_out);

}  // namespace fsdkr
