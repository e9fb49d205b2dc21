/* N-API binding of oracle/cpu/libblscpu.so -- TEST INFRASTRUCTURE (the CPU row of
 * tests/node/gossip_bench.js), never part of the product path.
 *
 * The C++ restatement of the verify path behind a Node interface, so the Node-level gossip
 * comparison runs both verifiers under the same callers (tests/node/CpuPoolVerifier.js restates
 * BlsMultiThreadWorkerPool's buffering and job packaging over it):
 *   init(abz, iso)                    curve constants (tests/node/build_cpu.py writes them)
 *   skToPk96(sks) -> Uint8Array       96-byte uncompressed pubkeys (affine x | y)
 *   verifyAsync(pk96, msgs32, sigs96, lens, jobs3, mode, threads, seed) -> Promise<Int32Array>
 *       blscpu_verify on a libuv pool thread: per job 1 valid, 0 invalid, < 0 error; the
 *       argument buffers stay referenced until the promise settles.
 * Built by tests/node/build_cpu.py (gcc, linked against oracle/cpu/libblscpu.so).
 */
#include <node_api.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int blscpu_init(const uint8_t* sswu_abz, const uint8_t* iso);
int blscpu_verify(const uint8_t* pk96, const uint8_t* msgs32, const uint8_t* sigs96, const uint32_t* sig_lens,
                  const uint32_t* jobs3, size_t njobs, int mode, int threads, uint64_t seed, int32_t* out);
int blscpu_sk_to_pk96(const uint8_t* sk32, size_t n, uint8_t* out96);

#define CHECK(env, call)                                   \
  do {                                                     \
    if ((call) != napi_ok) {                               \
      napi_throw_error((env), NULL, "blscpu: N-API call"); \
      return NULL;                                         \
    }                                                      \
  } while (0)

static int get_bytes(napi_env env, napi_value v, uint8_t** data, size_t* len) {
  napi_typedarray_type t;
  napi_value ab;
  size_t off;
  void* p;
  if (napi_get_typedarray_info(env, v, &t, len, &p, &ab, &off) != napi_ok) return -1;
  if (t == napi_uint32_array) *len *= 4;
  *data = (uint8_t*)p;
  return 0;
}

static napi_value js_init(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2], out;
  uint8_t *abz, *iso;
  size_t la, li;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 2 || get_bytes(env, argv[0], &abz, &la) || get_bytes(env, argv[1], &iso, &li) || la != 288 ||
      li != 15 * 96) {
    napi_throw_error(env, NULL, "blscpu.init(abz[288], iso[1440])");
    return NULL;
  }
  CHECK(env, napi_create_int32(env, blscpu_init(abz, iso), &out));
  return out;
}

static napi_value js_sk_to_pk96(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], ab, out;
  uint8_t* sks;
  size_t len;
  void* dst;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 1 || get_bytes(env, argv[0], &sks, &len)) {
    napi_throw_error(env, NULL, "blscpu.skToPk96(sks)");
    return NULL;
  }
  CHECK(env, napi_create_arraybuffer(env, 96 * (len / 32), &dst, &ab));
  blscpu_sk_to_pk96(sks, len / 32, (uint8_t*)dst);
  CHECK(env, napi_create_typedarray(env, napi_uint8_array, 96 * (len / 32), ab, 0, &out));
  return out;
}

enum { NBUF = 5 };
typedef struct {
  napi_async_work work;
  napi_deferred deferred;
  napi_ref refs[NBUF];
  uint8_t* buf[NBUF];
  size_t njobs;
  int mode, threads, rc;
  uint64_t seed;
  int32_t* out;
} verify_req;

static void verify_execute(napi_env env, void* data) {
  (void)env;
  verify_req* r = (verify_req*)data;
  r->rc = blscpu_verify(r->buf[0], r->buf[1], r->buf[2], (const uint32_t*)r->buf[3], (const uint32_t*)r->buf[4],
                        r->njobs, r->mode, r->threads, r->seed, r->out);
}

static void verify_complete(napi_env env, napi_status status, void* data) {
  verify_req* r = (verify_req*)data;
  if (status == napi_ok && r->rc == 0) {
    napi_value ab, arr;
    void* dst;
    napi_create_arraybuffer(env, 4 * (r->njobs ? r->njobs : 1), &dst, &ab);
    memcpy(dst, r->out, 4 * r->njobs);
    napi_create_typedarray(env, napi_int32_array, r->njobs, ab, 0, &arr);
    napi_resolve_deferred(env, r->deferred, arr);
  } else {
    napi_value msg, err;
    napi_create_string_utf8(env, "blscpu_verify failed", NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, NULL, msg, &err);
    napi_reject_deferred(env, r->deferred, err);
  }
  for (int i = 0; i < NBUF; ++i) napi_delete_reference(env, r->refs[i]);
  napi_delete_async_work(env, r->work);
  free(r->out);
  free(r);
}

static napi_value js_verify_async(napi_env env, napi_callback_info info) {
  size_t argc = 8;
  napi_value argv[8], promise, name;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 8) {
    napi_throw_error(env, NULL, "blscpu.verifyAsync(pk96, msgs, sigs, lens, jobs3, mode, threads, seed)");
    return NULL;
  }
  verify_req* r = (verify_req*)calloc(1, sizeof(verify_req));
  size_t len[NBUF];
  for (int i = 0; i < NBUF; ++i) {
    if (get_bytes(env, argv[i], &r->buf[i], &len[i])) {
      free(r);
      napi_throw_error(env, NULL, "blscpu.verifyAsync: typed arrays expected");
      return NULL;
    }
  }
  double seed = 0;
  napi_get_value_int32(env, argv[5], &r->mode);
  napi_get_value_int32(env, argv[6], &r->threads);
  napi_get_value_double(env, argv[7], &seed);
  r->seed = (uint64_t)seed;
  r->njobs = len[4] / 12;
  r->out = (int32_t*)calloc(r->njobs ? r->njobs : 1, 4);
  for (int i = 0; i < NBUF; ++i) CHECK(env, napi_create_reference(env, argv[i], 1, &r->refs[i]));
  CHECK(env, napi_create_promise(env, &r->deferred, &promise));
  CHECK(env, napi_create_string_utf8(env, "blscpu.verify", NAPI_AUTO_LENGTH, &name));
  CHECK(env, napi_create_async_work(env, NULL, name, verify_execute, verify_complete, r, &r->work));
  CHECK(env, napi_queue_async_work(env, r->work));
  return promise;
}

static napi_value init_module(napi_env env, napi_value exports) {
  napi_property_descriptor d[] = {
      {"init", NULL, js_init, NULL, NULL, NULL, napi_default, NULL},
      {"skToPk96", NULL, js_sk_to_pk96, NULL, NULL, NULL, napi_default, NULL},
      {"verifyAsync", NULL, js_verify_async, NULL, NULL, NULL, napi_default, NULL},
  };
  napi_define_properties(env, exports, sizeof(d) / sizeof(d[0]), d);
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init_module)
