// Batched RefreshMessage::collect verification: the first-error mapping
// (fsdkr_collect_first_error: the reference's check order) and the C ABI of the
// prestart / prepare / launch / finish stages (collect_prestart.cpp,
// collect_prepare.cpp, collect_launch.cpp; shared declarations in collect.hpp).
//
// One call verifies one or many independent collect() sessions in ONE device
// pass: the sessions' pairs, receivers, messages and joins are concatenated
// into a single image (little-endian u32 limbs, one fixed width per field);
// every descriptor addresses rows of that image.
//
// Reference: /root/reference/src/refresh_message.rs:321-467 (collect),
// :147-191 (validate_collect).
#include "collect.hpp"

namespace fsdkr {

void free_collect_plan(Ctx* c) {
  delete reinterpret_cast<CollectPlan*>(c->plan);
  c->plan = nullptr;
}

void free_ga_pre(Ctx* c) {
  GaPre* g = reinterpret_cast<GaPre*>(c->ga_pre);
  if (g && g->done) (void)hipEventDestroy(g->done);
  if (g && g->ga_setup) (void)hipEventDestroy(g->ga_setup);
  if (g && g->ga_rows_up) (void)hipEventDestroy(g->ga_rows_up);
  if (g && g->fb_done) (void)hipEventDestroy(g->fb_done);
  if (g && g->fb_setup) (void)hipEventDestroy(g->fb_setup);
  if (g && g->ck_done) (void)hipEventDestroy(g->ck_done);
  if (g && g->tz_done) (void)hipEventDestroy(g->tz_done);
  if (g && g->comb_done) (void)hipEventDestroy(g->comb_done);
  delete g;
  c->ga_pre = nullptr;
}

int first_error_impl(const fsdkr_collect_batch* b, const fsdkr_verdicts* v, fsdkr_error* e) {
  memset(e, 0, sizeof *e);
  const uint32_t R = b->n_refresh, J = b->n_join, n = R + J;
  // validate_collect (refresh_message.rs:147-191)
  if (R <= b->t) {
    e->variant = FSDKR_ERR_PARTIES_THRESHOLD_VIOLATION;
    e->f[0] = b->t;
    e->f[1] = R;
    return FSDKR_OK;
  }
  if (b->msg_lens) {
    const uint32_t ref = b->msg_lens[0];
    for (uint32_t k = 0; k < R; ++k) {
      const uint32_t* l = b->msg_lens + 3 * (size_t)k;
      if (!(l[0] == ref && l[1] == ref && l[2] == ref)) {
        e->variant = FSDKR_ERR_SIZE_MISMATCH;
        e->f[0] = k;
        e->f[1] = l[0];
        e->f[2] = l[1];
        e->f[3] = l[2];
        return FSDKR_OK;
      }
    }
    if (ref < n) {  // points_committed_vec[i] indexed past its end (:182); the host
                    // layer checks message 0's first `ref` shares before this panic
      e->panic = 1;
      e->variant = FSDKR_ERR_PUBLIC_SHARE_VALIDATION;
      return FSDKR_OK;
    }
  }
  if (!v) return FSDKR_E_ARG;
  if (v->cap_pairs < R * n || v->cap_msgs < R + J || (J && (!v->dlog || v->cap_joins < J))) return FSDKR_E_ARG;
  for (uint32_t k = 0; k < R; ++k)
    for (uint32_t i = 0; i < n; ++i) {
      const uint8_t f = v->feldman[(size_t)k * n + i];
      if (f & 2) {   // empty commitment vector: curv's unwrap panics
        e->panic = 1;
        e->variant = FSDKR_ERR_PUBLIC_SHARE_VALIDATION;
        return FSDKR_OK;
      }
      if (!(f & 1)) {
        e->variant = FSDKR_ERR_PUBLIC_SHARE_VALIDATION;
        return FSDKR_OK;
      }
    }
  // PDL then range, per (k, i)  (:330-350)
  for (uint32_t k = 0; k < R; ++k)
    for (uint32_t i = 0; i < n; ++i) {
      if (b->recv_avail && i >= b->recv_avail) {   // local_key.paillier_key_vec[i] out of bounds (:334)
        e->panic = 1;
        e->variant = FSDKR_ERR_PDL_W_SLACK_PROOF;
        return FSDKR_OK;
      }
      const uint8_t d = v->pdl[(size_t)k * n + i];
      if (d & 8) {
        e->panic = 1;
        e->variant = FSDKR_ERR_PDL_W_SLACK_PROOF;
        return FSDKR_OK;
      }
      if ((d & 7) != 7) {
        e->variant = FSDKR_ERR_PDL_W_SLACK_PROOF;
        e->f[0] = d & 1;
        e->f[1] = (d >> 1) & 1;
        e->f[2] = (d >> 2) & 1;
        return FSDKR_OK;
      }
      if (b->range_lens && i >= b->range_lens[k]) {   // range_proofs[i] out of bounds (:342)
        e->panic = 1;
        e->variant = FSDKR_ERR_RANGE_PROOF;
        e->f[0] = i;
        return FSDKR_OK;
      }
      if (v->range[(size_t)k * n + i] & 2) {   // a negative Alice exponent (host layer)
        e->panic = 1;
        e->variant = FSDKR_ERR_RANGE_PROOF;
        e->f[0] = i;
        return FSDKR_OK;
      }
      if (!(v->range[(size_t)k * n + i] & 1)) {
        e->variant = FSDKR_ERR_RANGE_PROOF;
        e->f[0] = i;
        return FSDKR_OK;
      }
    }
  // ring-Pedersen: refresh then join (:353-365)
  for (uint32_t m = 0; m < R + J; ++m) {
    if (v->ped[m] & 2) {
      e->panic = 1;
      e->variant = FSDKR_ERR_RING_PEDERSEN_PROOF;
      return FSDKR_OK;
    }
    if (!(v->ped[m] & 1)) {
      e->variant = FSDKR_ERR_RING_PEDERSEN_PROOF;
      return FSDKR_OK;
    }
  }
  const uint32_t ckl = b->ckl ? b->ckl : b->nl;
  // correct key + modulus size per refresh message (:375-396)
  for (uint32_t m = 0; m < R; ++m) {
    const uint32_t pi = b->party_index[m];
    if (v->ck[m] & 2) {   // sigma_vec[i] out of bounds in zk-paillier's verify
      e->panic = 1;
      e->variant = FSDKR_ERR_PAILLIER_VERIFICATION;
      e->f[0] = pi;
      return FSDKR_OK;
    }
    if (!(v->ck[m] & 1)) {
      e->variant = FSDKR_ERR_PAILLIER_VERIFICATION;
      e->f[0] = pi;
      return FSDKR_OK;
    }
    const uint32_t bits = hbn::bitlen(b->ck_n + (size_t)m * ckl, ckl);
    if (bits > b->key_bits || bits < b->key_bits - 1) {
      e->variant = FSDKR_ERR_MODULI_TOO_SMALL;
      e->f[0] = pi;
      e->f[1] = bits;
      return FSDKR_OK;
    }
    e->keys_applied = m + 1;
  }
  // joins (:398-437)
  for (uint32_t j = 0; j < J; ++j) {
    const uint32_t pi = b->party_index[R + j];
    if (pi == 0) {
      e->variant = FSDKR_ERR_NEW_PARTY_UNASSIGNED_INDEX;
      return FSDKR_OK;
    }
    if (v->ck[R + j] & 2) {
      e->panic = 1;
      e->variant = FSDKR_ERR_PAILLIER_VERIFICATION;
      e->f[0] = pi;
      return FSDKR_OK;
    }
    if (!(v->ck[R + j] & 1)) {
      e->variant = FSDKR_ERR_PAILLIER_VERIFICATION;
      e->f[0] = pi;
      return FSDKR_OK;
    }
    if (v->dlog[j] & 4) {   // a negative DLog response y (host layer)
      e->panic = 1;
      e->variant = FSDKR_ERR_DLOG_PROOF_VALIDATION;
      e->f[0] = pi;
      return FSDKR_OK;
    }
    if ((v->dlog[j] & 3) != 3) {
      e->variant = FSDKR_ERR_DLOG_PROOF_VALIDATION;
      e->f[0] = pi;
      return FSDKR_OK;
    }
    const uint32_t bits = hbn::bitlen(b->ck_n + (size_t)(R + j) * ckl, ckl);
    if (bits > b->key_bits || bits < b->key_bits - 1) {
      e->variant = FSDKR_ERR_MODULI_TOO_SMALL;
      e->f[0] = pi;
      e->f[1] = bits;
      return FSDKR_OK;
    }
    e->keys_applied = R + j + 1;
  }
  e->variant = FSDKR_ERR_NONE;
  return FSDKR_OK;
}

}  // namespace fsdkr

extern "C" {

int fsdkr_collect_prepare_multi(fsdkr_ctx* ctx, const fsdkr_collect_batch* batches, uint32_t count) {
  fsdkr::Ctx* c = reinterpret_cast<fsdkr::Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  return fsdkr::collect_prepare_impl(c, batches, count);
}

int fsdkr_collect_prepare(fsdkr_ctx* ctx, const fsdkr_collect_batch* batch) {
  return fsdkr_collect_prepare_multi(ctx, batch, 1);
}

int fsdkr_collect_prestart(fsdkr_ctx* ctx, const fsdkr_collect_batch* batch) {
  fsdkr::Ctx* c = reinterpret_cast<fsdkr::Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  return fsdkr::collect_prestart_impl(c, batch, 1);
}

int fsdkr_collect_prestart_multi(fsdkr_ctx* ctx, const fsdkr_collect_batch* batches, uint32_t count) {
  fsdkr::Ctx* c = reinterpret_cast<fsdkr::Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  return fsdkr::collect_prestart_impl(c, batches, count);
}

int fsdkr_collect_prestart_rp(fsdkr_ctx* ctx, const fsdkr_collect_batch* batches, uint32_t count) {
  fsdkr::Ctx* c = reinterpret_cast<fsdkr::Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  return fsdkr::collect_prestart_rp_impl(c, batches, count);
}

int fsdkr_collect_launch(fsdkr_ctx* ctx) {
  fsdkr::Ctx* c = reinterpret_cast<fsdkr::Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  return fsdkr::collect_launch_impl(c);
}

int fsdkr_collect_finish_multi(fsdkr_ctx* ctx, fsdkr_verdicts* out, uint32_t count) {
  fsdkr::Ctx* c = reinterpret_cast<fsdkr::Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  return fsdkr::collect_finish_impl(c, out, count);
}

int fsdkr_collect_finish(fsdkr_ctx* ctx, fsdkr_verdicts* out) { return fsdkr_collect_finish_multi(ctx, out, 1); }

int fsdkr_collect_run(fsdkr_ctx* ctx, fsdkr_verdicts* out) {
  int rc = fsdkr_collect_launch(ctx);
  return rc ? rc : fsdkr_collect_finish(ctx, out);
}

int fsdkr_verify_collect_multi(fsdkr_ctx* ctx, const fsdkr_collect_batch* batches, uint32_t count,
                               fsdkr_verdicts* out) {
  if (!ctx || !batches || !out || count == 0) return FSDKR_E_ARG;
  int rc = fsdkr_collect_prepare_multi(ctx, batches, count);
  if (!rc) rc = fsdkr_collect_launch(ctx);
  if (!rc) rc = fsdkr_collect_finish_multi(ctx, out, count);
  return rc;
}

int fsdkr_verify_collect(fsdkr_ctx* ctx, const fsdkr_collect_batch* batch, fsdkr_verdicts* out) {
  return fsdkr_verify_collect_multi(ctx, batch, 1, out);
}

int fsdkr_collect_first_error(const fsdkr_collect_batch* batch, const fsdkr_verdicts* verdicts, fsdkr_error* out) {
  if (!batch || !out) return FSDKR_E_ARG;
  return fsdkr::first_error_impl(batch, verdicts, out);
}

int fsdkr_collect_first_error_multi(const fsdkr_collect_batch* batches, const fsdkr_verdicts* verdicts, uint32_t count,
                                    fsdkr_error* out) {
  if (count && (!batches || !verdicts || !out)) return FSDKR_E_ARG;
  for (uint32_t s = 0; s < count; ++s) {
    const int rc = fsdkr::first_error_impl(batches + s, verdicts + s, out + s);
    if (rc) return rc;
  }
  return FSDKR_OK;
}

}  // extern "C"
