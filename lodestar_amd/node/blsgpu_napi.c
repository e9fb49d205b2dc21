/*
 * blsgpu.node — N-API binding of libblsgpu.so for Node (the reference's own runtime).
 *
 * Exposes the C-ABI (include/blsgpu.h) to JavaScript; BlsGpuVerifier.js builds the
 * IBlsVerifier (packages/beacon-node/src/chain/bls/interface.ts:20-46) on top.
 * Verification goes through bgv_verify_async: the library's dispatcher threads run it and
 * hand the completion to the main thread through a napi_threadsafe_function, which
 * resolves the Promise, like the reference's worker round trip
 * (multithread/index.ts:290-381).  No libuv pool thread is held while a batch runs.
 *
 * Lifetime: the ctx value is an external over a small wrapper.  close(ctx) is idempotent:
 * it closes the library context (queued and in-flight verifies complete first, later
 * calls reject with QUEUE_ABORTED) but does not free it; the memory is released by the
 * external's finalizer, which cannot run while a verify holds a reference to the ctx.
 *
 *   init(devices?: number[]) -> ctx
 *   pubkeysPut(ctx, firstIndex, keys: Uint8Array, fmt: 48 | 96)
 *   pubkeysPutAsync(ctx, firstIndex, keys, fmt) -> Promise<void>  (on a libuv pool thread)
 *   keygen(ctx, sks: Uint8Array, cacheFirst: number) -> Uint8Array (48-B pubkeys)
 *   sign(ctx, sks: Uint8Array, msgs: Uint8Array) -> Uint8Array (96-B signatures)
 *   verify(ctx, jobs: {sets: {pkIndices: Uint32Array | pkBytes: Uint8Array (n x 96),
 *                             msg: Uint8Array, sig: Uint8Array}[], batchable: boolean}[],
 *          mode: 0 | 1) -> Promise<Int32Array>   (1 valid, 0 invalid, -code error)
 *   strerror(code) -> string
 *   close(ctx)
 * SURVEY 8(f) entry points and parity hooks (synchronous):
 *   aggregatePubkeys(ctx, indices: Uint32Array) -> Uint8Array (96-B uncompressed)
 *   hashToG2(ctx, msg: Uint8Array) -> Uint8Array (192-B uncompressed)
 *   pubkeysValidate(ctx, keys48) -> {status: Int32Array, uncompressed: Uint8Array}
 *   aggregateSignatures(ctx, aggregates: Uint8Array[][]) -> {status: Int32Array, sigs: Uint8Array}
 *   depositsVerify(ctx, keys48, msgs32, sigs96) -> Int32Array (1 | 0)
 */
#include <node_api.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/blsgpu.h"

#define CHECK(env, x)                                         \
  do {                                                        \
    if ((x) != napi_ok) {                                     \
      napi_throw_error((env), NULL, "blsgpu: N-API failure"); \
      return NULL;                                            \
    }                                                         \
  } while (0)

static napi_value throw_code(napi_env env, int rc) {
  napi_throw_error(env, NULL, bgv_strerror(rc));
  return NULL;
}

typedef struct {
  bgv_ctx* c;
  int closed;                    /* close() was called: every entry point rejects */
  uint32_t inflight;             /* async verifies not yet completed */
  napi_threadsafe_function tsfn; /* completions from the dispatcher threads */
  int tsfn_released;             /* released by close() or finalized by the runtime */
  int owners;                    /* the ctx external and the tsfn: freed when both are gone */
} addon_ctx;

static void addon_unref(addon_ctx* a) {
  if (--a->owners == 0) {
    bgv_destroy(a->c);
    free(a);
  }
}

static addon_ctx* get_actx(napi_env env, napi_value v) {
  void* p = NULL;
  if (napi_get_value_external(env, v, &p) != napi_ok) return NULL;
  return (addon_ctx*)p;
}

/* the library context of an open addon context, else NULL (the caller throws) */
static bgv_ctx* get_ctx(napi_env env, napi_value v) {
  addon_ctx* a = get_actx(env, v);
  return a && !a->closed ? a->c : NULL;
}

#define OPEN_CTX(env, v, ctx)                                 \
  bgv_ctx* ctx = get_ctx((env), (v));                         \
  do {                                                        \
    if (!ctx) return throw_code((env), -BGV_E_CLOSED);        \
  } while (0)

static int get_bytes(napi_env env, napi_value v, uint8_t** data, size_t* len) {
  napi_typedarray_type t;
  size_t n, off;
  void* d;
  napi_value ab;
  if (napi_get_typedarray_info(env, v, &t, &n, &d, &ab, &off) != napi_ok) return -1;
  if (t == napi_uint8_array) {
    *data = (uint8_t*)d;
    *len = n;
    return 0;
  }
  if (t == napi_uint32_array) {
    *data = (uint8_t*)d;
    *len = n * 4;
    return 0;
  }
  return -1;
}

typedef struct {
  addon_ctx* actx;
  napi_ref ctx_ref; /* keeps the ctx external (and its finalizer) alive */
  bgv_job* jobs;
  size_t njobs;
  bgv_set* sets;
  size_t nsets;
  int mode;
  int32_t* codes;
  bgv_stats stats;
  int rc;
  napi_deferred deferred;
  napi_ref* refs; /* keep every input buffer alive until completion */
  size_t nrefs;
} verify_req;

static void verify_call_js(napi_env env, napi_value js_cb, void* context, void* data);
static void addon_finalize(napi_env env, void* data, void* hint);
static void tsfn_finalized(napi_env env, void* data, void* hint);

static napi_value js_init(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  int devs[64];
  int ndev = 0;
  if (argc >= 1) {
    bool is_arr = false;
    napi_is_array(env, argv[0], &is_arr);
    if (is_arr) {
      uint32_t n = 0;
      napi_get_array_length(env, argv[0], &n);
      for (uint32_t i = 0; i < n && i < 64; ++i) {
        napi_value e;
        napi_get_element(env, argv[0], i, &e);
        napi_get_value_int32(env, e, &devs[ndev++]);
      }
    }
  }
  bgv_ctx* ctx = NULL;
  int rc = bgv_init(ndev ? devs : NULL, ndev, &ctx);
  if (rc) return throw_code(env, rc);
  addon_ctx* a = (addon_ctx*)calloc(1, sizeof(addon_ctx));
  a->c = ctx;
  a->owners = 2;
  napi_value out, name;
  if (napi_create_string_utf8(env, "blsgpu.verify.done", NAPI_AUTO_LENGTH, &name) != napi_ok ||
      napi_create_threadsafe_function(env, NULL, NULL, name, 0, 1, a, tsfn_finalized, NULL, verify_call_js,
                                      &a->tsfn) != napi_ok ||
      napi_unref_threadsafe_function(env, a->tsfn) != napi_ok ||
      napi_create_external(env, a, addon_finalize, NULL, &out) != napi_ok) {
    bgv_destroy(ctx);
    free(a);
    napi_throw_error(env, NULL, "blsgpu: N-API failure");
    return NULL;
  }
  return out;
}

/* close(ctx): idempotent; the library drains queued and in-flight verifies (their
 * completions still resolve), and every later call rejects with QUEUE_ABORTED. */
static napi_value js_close(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* a = get_actx(env, argv[0]);
  if (a && !a->closed) {
    a->closed = 1;
    bgv_close(a->c);  /* every queued completion has been handed to the tsfn */
    if (!a->tsfn_released) {
      a->tsfn_released = 1;
      napi_release_threadsafe_function(a->tsfn, napi_tsfn_release);  /* delivers them, then finalizes */
    }
  }
  return NULL;
}

static napi_value js_strerror(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], out;
  int32_t code = 0;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  napi_get_value_int32(env, argv[0], &code);
  CHECK(env, napi_create_string_utf8(env, bgv_strerror(code), NAPI_AUTO_LENGTH, &out));
  return out;
}

static napi_value js_pubkeys_put(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  OPEN_CTX(env, argv[0], ctx);
  uint32_t first = 0;
  int32_t fmt = 48;
  uint8_t* keys;
  size_t len;
  napi_get_value_uint32(env, argv[1], &first);
  if (get_bytes(env, argv[2], &keys, &len)) return throw_code(env, -BGV_E_ARG);
  napi_get_value_int32(env, argv[3], &fmt);
  int rc = bgv_pubkeys_put(ctx, first, keys, len / (size_t)fmt, fmt);
  if (rc) return throw_code(env, rc);
  return NULL;
}

/* pubkeysPutAsync(ctx, firstIndex, keys, fmt) -> Promise<void>: bgv_pubkeys_put on a libuv pool
 * thread, so a validator-set growth (EpochContext.addPubkey, epochContext.ts:702-705) never
 * blocks the event loop; the library decodes into staging memory without holding up running
 * verifies.  Rejects with an Error whose .bgvCode is the negative library code (-BGV_E_ARG for
 * a gap in the indices: nothing was written; a BLST code: the run was committed with the
 * undecodable indices marked). */
typedef struct {
  napi_async_work work;
  napi_deferred deferred;
  napi_ref ctx_ref, keys_ref;
  bgv_ctx* c;
  uint32_t first;
  const uint8_t* keys;
  size_t n;
  int fmt, rc;
} put_req;

static void put_execute(napi_env env, void* data) {
  (void)env;
  put_req* r = (put_req*)data;
  r->rc = bgv_pubkeys_put(r->c, r->first, r->keys, r->n, r->fmt);
}

static void put_complete(napi_env env, napi_status status, void* data) {
  put_req* r = (put_req*)data;
  if (status == napi_ok && r->rc == 0) {
    napi_value undef;
    napi_get_undefined(env, &undef);
    napi_resolve_deferred(env, r->deferred, undef);
  } else {
    const int rc = status == napi_ok ? r->rc : -BGV_E_ARG;
    napi_value msg, err, code;
    napi_create_string_utf8(env, bgv_strerror(rc), NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, NULL, msg, &err);
    napi_create_int32(env, rc, &code);
    napi_set_named_property(env, err, "bgvCode", code);
    napi_reject_deferred(env, r->deferred, err);
  }
  napi_delete_reference(env, r->ctx_ref);
  napi_delete_reference(env, r->keys_ref);
  napi_delete_async_work(env, r->work);
  free(r);
}

static napi_value js_pubkeys_put_async(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4], promise, name;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  OPEN_CTX(env, argv[0], ctx);
  uint8_t* keys;
  size_t len;
  uint32_t first = 0;
  int32_t fmt = 48;
  napi_get_value_uint32(env, argv[1], &first);
  if (get_bytes(env, argv[2], &keys, &len)) return throw_code(env, -BGV_E_ARG);
  napi_get_value_int32(env, argv[3], &fmt);
  if (fmt != 48 && fmt != 96) return throw_code(env, -BGV_E_ARG);
  put_req* r = (put_req*)calloc(1, sizeof(put_req));
  r->c = ctx;
  r->first = first;
  r->keys = keys;
  r->n = len / (size_t)fmt;
  r->fmt = fmt;
  if (napi_create_promise(env, &r->deferred, &promise) != napi_ok ||
      napi_create_reference(env, argv[0], 1, &r->ctx_ref) != napi_ok ||
      napi_create_reference(env, argv[2], 1, &r->keys_ref) != napi_ok ||
      napi_create_string_utf8(env, "blsgpu.pubkeysPut", NAPI_AUTO_LENGTH, &name) != napi_ok ||
      napi_create_async_work(env, NULL, name, put_execute, put_complete, r, &r->work) != napi_ok ||
      napi_queue_async_work(env, r->work) != napi_ok) {
    napi_throw_error(env, NULL, "blsgpu: N-API failure");
    return NULL;
  }
  return promise;
}

static napi_value js_keygen(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3], ab, out;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  OPEN_CTX(env, argv[0], ctx);
  uint8_t* sks;
  size_t len;
  int64_t first = -1;
  if (get_bytes(env, argv[1], &sks, &len)) return throw_code(env, -BGV_E_ARG);
  napi_get_value_int64(env, argv[2], &first);
  void* dst;
  CHECK(env, napi_create_arraybuffer(env, 48 * (len / 32), &dst, &ab));
  int rc = bgv_keygen(ctx, sks, len / 32, first, (uint8_t*)dst);
  if (rc) return throw_code(env, rc);
  CHECK(env, napi_create_typedarray(env, napi_uint8_array, 48 * (len / 32), ab, 0, &out));
  return out;
}

static napi_value js_sign(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3], ab, out;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  OPEN_CTX(env, argv[0], ctx);
  uint8_t *sks, *msgs;
  size_t l1, l2;
  if (get_bytes(env, argv[1], &sks, &l1) || get_bytes(env, argv[2], &msgs, &l2) || l1 != l2)
    return throw_code(env, -BGV_E_ARG);
  void* dst;
  CHECK(env, napi_create_arraybuffer(env, 96 * (l1 / 32), &dst, &ab));
  int rc = bgv_sign(ctx, sks, msgs, l1 / 32, (uint8_t*)dst);
  if (rc) return throw_code(env, rc);
  CHECK(env, napi_create_typedarray(env, napi_uint8_array, 96 * (l1 / 32), ab, 0, &out));
  return out;
}

/* ---- SURVEY 8(f) entry points and parity hooks (synchronous: low volume) ---- */

static napi_value new_bytes(napi_env env, size_t n, void** dst) {
  napi_value ab, out;
  if (napi_create_arraybuffer(env, n, dst, &ab) != napi_ok) return NULL;
  if (napi_create_typedarray(env, napi_uint8_array, n, ab, 0, &out) != napi_ok) return NULL;
  return out;
}

static napi_value new_int32s(napi_env env, const int32_t* src, size_t n) {
  napi_value ab, out;
  void* dst;
  if (napi_create_arraybuffer(env, 4 * n, &dst, &ab) != napi_ok) return NULL;
  if (n) memcpy(dst, src, 4 * n);
  if (napi_create_typedarray(env, napi_int32_array, n, ab, 0, &out) != napi_ok) return NULL;
  return out;
}

/* aggregatePubkeys(ctx, indices: Uint32Array) -> Uint8Array(96): PublicKey.aggregate +
 * toBytes(uncompressed) over cached keys (chain/bls/utils.ts:5-16). */
static napi_value js_aggregate_pubkeys(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  OPEN_CTX(env, argv[0], ctx);
  uint8_t* idx;
  size_t len;
  if (get_bytes(env, argv[1], &idx, &len) || len % 4) return throw_code(env, -BGV_E_ARG);
  void* dst;
  napi_value out = new_bytes(env, 96, &dst);
  if (!out) return throw_code(env, -BGV_E_ARG);
  int rc = bgv_aggregate_pubkeys(ctx, (const uint32_t*)idx, len / 4, (uint8_t*)dst);
  if (rc) return throw_code(env, rc);
  return out;
}

/* hashToG2(ctx, msg: Uint8Array) -> Uint8Array(192) uncompressed (x.c1|x.c0|y.c1|y.c0) */
static napi_value js_hash_to_g2(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  OPEN_CTX(env, argv[0], ctx);
  uint8_t* msg;
  size_t len;
  if (get_bytes(env, argv[1], &msg, &len)) return throw_code(env, -BGV_E_ARG);
  uint32_t l32 = (uint32_t)len;
  void* dst;
  napi_value out = new_bytes(env, 192, &dst);
  if (!out) return throw_code(env, -BGV_E_ARG);
  int rc = bgv_hash_to_g2(ctx, msg, &l32, 1, (uint8_t*)dst);
  if (rc) return throw_code(env, rc);
  return out;
}

/* pubkeysValidate(ctx, keys48: Uint8Array (n x 48)) -> {status: Int32Array (0 | -BLST code),
 * uncompressed: Uint8Array (n x 96)}: PublicKey.fromBytes(pk, affine, validate=true) per key
 * (state-transition/src/block/processDeposit.ts:64). */
static napi_value js_pubkeys_validate(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  OPEN_CTX(env, argv[0], ctx);
  uint8_t* keys;
  size_t len;
  if (get_bytes(env, argv[1], &keys, &len) || len % 48) return throw_code(env, -BGV_E_ARG);
  const size_t n = len / 48;
  int32_t* st = (int32_t*)calloc(n ? n : 1, sizeof(int32_t));
  void* dst;
  napi_value recs = new_bytes(env, 96 * n, &dst);
  if (!recs) {
    free(st);
    return throw_code(env, -BGV_E_ARG);
  }
  int rc = bgv_pubkeys_validate(ctx, keys, n, st, (uint8_t*)dst);
  if (rc) {
    free(st);
    return throw_code(env, rc);
  }
  napi_value out, status = new_int32s(env, st, n);
  free(st);
  CHECK(env, napi_create_object(env, &out));
  CHECK(env, napi_set_named_property(env, out, "status", status));
  CHECK(env, napi_set_named_property(env, out, "uncompressed", recs));
  return out;
}

/* aggregateSignatures(ctx, aggregates: Uint8Array[][]) -> {status: Int32Array, sigs: Uint8Array
 * (naggs x 96 compressed)}: Signature.aggregate over validated signatures, one entry per
 * op-pool aggregate (chain/opPools/attestationPool.ts:184-187 and siblings). */
static napi_value js_aggregate_signatures(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  OPEN_CTX(env, argv[0], ctx);
  uint32_t naggs = 0;
  if (napi_get_array_length(env, argv[1], &naggs) != napi_ok) return throw_code(env, -BGV_E_ARG);
  uint32_t* counts = (uint32_t*)calloc(naggs ? naggs : 1, sizeof(uint32_t));
  size_t total = 0;
  for (uint32_t a = 0; a < naggs; ++a) {
    napi_value agg;
    napi_get_element(env, argv[1], a, &agg);
    if (napi_get_array_length(env, agg, &counts[a]) != napi_ok) {
      free(counts);
      return throw_code(env, -BGV_E_ARG);
    }
    total += counts[a];
  }
  /* records are zero-padded to 96 B; lens carries the received size (BLST_INVALID_SIZE) */
  uint8_t* raw = (uint8_t*)calloc(total ? total : 1, 96);
  uint32_t* lens = (uint32_t*)calloc(total ? total : 1, sizeof(uint32_t));
  int32_t* st = (int32_t*)calloc(naggs ? naggs : 1, sizeof(int32_t));
  size_t k = 0;
  int bad = 0;
  for (uint32_t a = 0; a < naggs && !bad; ++a) {
    napi_value agg;
    napi_get_element(env, argv[1], a, &agg);
    for (uint32_t i = 0; i < counts[a]; ++i, ++k) {
      napi_value s;
      uint8_t* d;
      size_t l;
      napi_get_element(env, agg, i, &s);
      if (get_bytes(env, s, &d, &l)) {
        bad = 1;
        break;
      }
      memcpy(raw + 96 * k, d, l < 96 ? l : 96);
      lens[k] = (uint32_t)l;
    }
  }
  void* dst;
  napi_value sigs = bad ? NULL : new_bytes(env, 96 * (size_t)naggs, &dst);
  int rc = sigs ? bgv_aggregate_signatures(ctx, raw, lens, counts, naggs, (uint8_t*)dst, st) : -BGV_E_ARG;
  napi_value status = rc ? NULL : new_int32s(env, st, naggs);
  free(raw);
  free(lens);
  free(counts);
  free(st);
  if (rc) return throw_code(env, rc);
  napi_value out;
  CHECK(env, napi_create_object(env, &out));
  CHECK(env, napi_set_named_property(env, out, "status", status));
  CHECK(env, napi_set_named_property(env, out, "sigs", sigs));
  return out;
}

/* depositsVerify(ctx, keys48, msgs32, sigs96) -> Int32Array (1 valid, 0 invalid): the
 * deposit signature check of processDeposit.ts:62-70. */
static napi_value js_deposits_verify(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  OPEN_CTX(env, argv[0], ctx);
  uint8_t *keys, *msgs, *sigs;
  size_t lk, lm, ls;
  if (get_bytes(env, argv[1], &keys, &lk) || get_bytes(env, argv[2], &msgs, &lm) ||
      get_bytes(env, argv[3], &sigs, &ls) || lk % 48 || lm != 32 * (lk / 48) || ls != 96 * (lk / 48))
    return throw_code(env, -BGV_E_ARG);
  const size_t n = lk / 48;
  int32_t* valid = (int32_t*)calloc(n ? n : 1, sizeof(int32_t));
  int rc = bgv_deposits_verify(ctx, keys, msgs, sigs, n, valid);
  napi_value out = rc ? NULL : new_int32s(env, valid, n);
  free(valid);
  if (rc) return throw_code(env, rc);
  return out;
}

/* ---- verify: bgv_verify_async + threadsafe completion + Promise ----------- */
static void free_req(napi_env env, verify_req* r) {
  for (size_t i = 0; i < r->nrefs; ++i) napi_delete_reference(env, r->refs[i]);
  if (r->ctx_ref) napi_delete_reference(env, r->ctx_ref);
  free(r->refs);
  free(r->jobs);
  free(r->sets);
  free(r->codes);
  free(r);
}

static void settle(napi_env env, verify_req* r) {
  if (r->rc) {
    napi_value err, msg;
    napi_create_string_utf8(env, bgv_strerror(r->rc), NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, NULL, msg, &err);
    napi_reject_deferred(env, r->deferred, err);
    return;
  }
  napi_value ab, arr;
  void* dst;
  napi_create_arraybuffer(env, 4 * r->njobs, &dst, &ab);
  memcpy(dst, r->codes, 4 * r->njobs);
  napi_create_typedarray(env, napi_int32_array, r->njobs, ab, 0, &arr);
  /* codes.stats: the call's BlsWorkResult-style counters (multithread/types.ts:24-36) */
  napi_value st, v;
  napi_create_object(env, &st);
  napi_create_double(env, (double)r->stats.batch_retries, &v);
  napi_set_named_property(env, st, "batchRetries", v);
  napi_create_double(env, (double)r->stats.batch_sigs_success, &v);
  napi_set_named_property(env, st, "batchSigsSuccess", v);
  napi_create_double(env, (double)r->stats.device_groups, &v);
  napi_set_named_property(env, st, "deviceGroups", v);
  napi_create_double(env, (double)r->stats.sets_verified, &v);
  napi_set_named_property(env, st, "setsVerified", v);
  napi_create_double(env, r->stats.device_ms, &v);
  napi_set_named_property(env, st, "deviceMs", v);
  napi_create_double(env, r->stats.wall_ms, &v);
  napi_set_named_property(env, st, "wallMs", v);
  napi_set_named_property(env, arr, "stats", st);
  napi_resolve_deferred(env, r->deferred, arr);
}

/* main thread: a verify finished on a dispatcher thread */
static void verify_call_js(napi_env env, napi_value js_cb, void* context, void* data) {
  (void)js_cb;
  (void)context;
  verify_req* r = (verify_req*)data;
  if (env) {
    addon_ctx* a = r->actx;
    settle(env, r);
    if (--a->inflight == 0 && !a->tsfn_released) napi_unref_threadsafe_function(env, a->tsfn);
    free_req(env, r);
  } else {
    /* environment teardown drained the queue: no JS to settle (the promise dies with the
     * environment) and no env for the references (they die with it too); free the heap part */
    free(r->refs);
    free(r->jobs);
    free(r->sets);
    free(r->codes);
    free(r);
  }
}

/* dispatcher thread (library): codes and stats are filled; hop to the main thread */
static void verify_done(void* user, int rc) {
  verify_req* r = (verify_req*)user;
  r->rc = rc;
  napi_call_threadsafe_function(r->actx->tsfn, r, napi_tsfn_nonblocking);
}

/* the runtime finalized the tsfn (after close() released it, or at environment teardown) */
static void tsfn_finalized(napi_env env, void* data, void* hint) {
  (void)env;
  (void)hint;
  addon_ctx* a = (addon_ctx*)data;
  a->tsfn_released = 1;
  addon_unref(a);
}

/* the ctx external was collected: no verify references it any more */
static void addon_finalize(napi_env env, void* data, void* hint) {
  (void)env;
  (void)hint;
  addon_ctx* a = (addon_ctx*)data;
  if (!a) return;
  if (!a->closed) {
    a->closed = 1;
    bgv_close(a->c);
  }
  if (!a->tsfn_released) {
    a->tsfn_released = 1;
    napi_release_threadsafe_function(a->tsfn, napi_tsfn_abort);
  }
  addon_unref(a);
}

static napi_value js_verify(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  addon_ctx* a = get_actx(env, argv[0]);
  if (!a || a->closed) { /* the Promise rejects (QUEUE_ABORTED), as every verify outcome is async */
    napi_deferred d;
    napi_value promise, err, msg;
    CHECK(env, napi_create_promise(env, &d, &promise));
    napi_create_string_utf8(env, bgv_strerror(-BGV_E_CLOSED), NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, NULL, msg, &err);
    napi_reject_deferred(env, d, err);
    return promise;
  }
  verify_req* r = (verify_req*)calloc(1, sizeof(verify_req));
  r->actx = a;
  int32_t mode = 0;
  if (argc >= 3) napi_get_value_int32(env, argv[2], &mode);
  r->mode = mode;
  uint32_t njobs = 0;
  napi_get_array_length(env, argv[1], &njobs);
  r->njobs = njobs;
  r->jobs = (bgv_job*)calloc(njobs ? njobs : 1, sizeof(bgv_job));
  r->codes = (int32_t*)calloc(njobs ? njobs : 1, sizeof(int32_t));
  size_t cap = 64;
  r->sets = (bgv_set*)calloc(cap, sizeof(bgv_set));
  size_t refcap = 256;
  r->refs = (napi_ref*)calloc(refcap, sizeof(napi_ref));
  for (uint32_t j = 0; j < njobs; ++j) {
    napi_value job, sets, bval;
    napi_get_element(env, argv[1], j, &job);
    napi_get_named_property(env, job, "sets", &sets);
    napi_get_named_property(env, job, "batchable", &bval);
    bool batchable = false;
    napi_get_value_bool(env, bval, &batchable);
    uint32_t ns = 0;
    napi_get_array_length(env, sets, &ns);
    r->jobs[j].first_set = (uint32_t)r->nsets;
    r->jobs[j].n_sets = ns;
    r->jobs[j].batchable = batchable;
    for (uint32_t k = 0; k < ns; ++k) {
      if (r->nsets == cap) {
        cap *= 2;
        r->sets = (bgv_set*)realloc(r->sets, cap * sizeof(bgv_set));
      }
      if (r->nrefs + 4 > refcap) {
        refcap *= 2;
        r->refs = (napi_ref*)realloc(r->refs, refcap * sizeof(napi_ref));
      }
      napi_value s, pk, msg, sig;
      napi_get_element(env, sets, k, &s);
      /* pkIndices (validator indices into the device cache) or pkBytes (n x 96-B uncompressed) */
      bool by_index = false;
      napi_has_named_property(env, s, "pkIndices", &by_index);
      napi_get_named_property(env, s, by_index ? "pkIndices" : "pkBytes", &pk);
      napi_get_named_property(env, s, "msg", &msg);
      napi_get_named_property(env, s, "sig", &sig);
      bgv_set* st = &r->sets[r->nsets++];
      memset(st, 0, sizeof(*st));
      uint8_t *pkd, *md, *sd;
      size_t pkl, ml, sl;
      if (get_bytes(env, pk, &pkd, &pkl) || get_bytes(env, msg, &md, &ml) || get_bytes(env, sig, &sd, &sl) ||
          ml != 32 || (!by_index && pkl % 96)) {
        free_req(env, r);
        return throw_code(env, -BGV_E_ARG);
      }
      if (by_index) {
        st->n_pk = (uint32_t)(pkl / 4);
        st->pk_indices = (const uint32_t*)pkd;
      } else {
        st->n_pk = (uint32_t)(pkl / 96);
        st->pk_bytes = pkd;
      }
      st->msg = md;
      st->sig = sd;
      st->sig_len = (uint32_t)sl;
      napi_create_reference(env, pk, 1, &r->refs[r->nrefs++]);
      napi_create_reference(env, msg, 1, &r->refs[r->nrefs++]);
      napi_create_reference(env, sig, 1, &r->refs[r->nrefs++]);
    }
  }
  napi_value promise;
  CHECK(env, napi_create_promise(env, &r->deferred, &promise));
  /* the ctx external stays alive (no finalizer) until this request completes */
  CHECK(env, napi_create_reference(env, argv[0], 1, &r->ctx_ref));
  if (a->inflight++ == 0) napi_ref_threadsafe_function(env, a->tsfn);
  int rc = bgv_verify_async(a->c, r->jobs, r->njobs, r->sets, r->nsets, r->mode, r->codes, &r->stats, verify_done, r);
  if (rc) { /* rejected before queueing (closed, bad arguments): settle now */
    r->rc = rc;
    settle(env, r);
    if (--a->inflight == 0) napi_unref_threadsafe_function(env, a->tsfn);
    free_req(env, r);
  }
  return promise;
}

#define METHOD_ATTR ((napi_property_attributes)(napi_writable | napi_enumerable | napi_configurable))

static napi_value init_module(napi_env env, napi_value exports) {
  napi_property_descriptor d[] = {
      {"init", NULL, js_init, NULL, NULL, NULL, METHOD_ATTR, NULL},
      {"close", NULL, js_close, NULL, NULL, NULL, METHOD_ATTR, NULL},
      {"strerror", NULL, js_strerror, NULL, NULL, NULL, METHOD_ATTR, NULL},
      {"pubkeysPut", NULL, js_pubkeys_put, NULL, NULL, NULL, METHOD_ATTR, NULL},
      {"pubkeysPutAsync", NULL, js_pubkeys_put_async, NULL, NULL, NULL, METHOD_ATTR, NULL},
      {"keygen", NULL, js_keygen, NULL, NULL, NULL, METHOD_ATTR, NULL},
      {"sign", NULL, js_sign, NULL, NULL, NULL, METHOD_ATTR, NULL},
      {"verify", NULL, js_verify, NULL, NULL, NULL, METHOD_ATTR, NULL},
      {"aggregatePubkeys", NULL, js_aggregate_pubkeys, NULL, NULL, NULL, METHOD_ATTR, NULL},
      {"hashToG2", NULL, js_hash_to_g2, NULL, NULL, NULL, METHOD_ATTR, NULL},
      {"pubkeysValidate", NULL, js_pubkeys_validate, NULL, NULL, NULL, METHOD_ATTR, NULL},
      {"aggregateSignatures", NULL, js_aggregate_signatures, NULL, NULL, NULL, METHOD_ATTR, NULL},
      {"depositsVerify", NULL, js_deposits_verify, NULL, NULL, NULL, METHOD_ATTR, NULL},
  };
  napi_define_properties(env, exports, sizeof(d) / sizeof(d[0]), d);
  napi_value n;
  napi_create_int32(env, bgv_device_count(), &n);
  napi_set_named_property(env, exports, "deviceCount", n);
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init_module)
