/*
 * brotli_amd.node -- Node-API binding of the brotli_amd C ABI (include/brotli_amd.h).
 *
 * This is the native half of the drop-in for countertype/brotli-lib's public surface
 * (package.json:7-23); index.js is the JavaScript half that keeps the reference's argument
 * handling and error messages.  Every function is synchronous on the JS thread, like the
 * reference's.  Result bytes are copied into a fresh Node Buffer and the library buffer
 * is released at once (mib_buf_free).
 */
#include <node_api.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/brotli_amd.h"

#define CHECK(env, call)                                   \
  do {                                                     \
    if ((call) != napi_ok) {                               \
      napi_throw_error((env), NULL, "brotli_amd: N-API"); \
      return NULL;                                         \
    }                                                      \
  } while (0)

static int get_bytes(napi_env env, napi_value v, const uint8_t **p, size_t *n) {
  bool is_typed = false, is_buf = false;
  napi_is_typedarray(env, v, &is_typed);
  if (is_typed) {
    napi_typedarray_type t;
    size_t len, off;
    void *data;
    napi_value ab;
    if (napi_get_typedarray_info(env, v, &t, &len, &data, &ab, &off) != napi_ok) return -1;
    size_t el = (t == napi_uint8_array || t == napi_int8_array || t == napi_uint8_clamped_array) ? 1 : 0;
    if (!el) return -1;
    *p = (const uint8_t *)data;
    *n = len;
    return 0;
  }
  napi_is_buffer(env, v, &is_buf);
  if (is_buf) {
    void *data;
    if (napi_get_buffer_info(env, v, &data, n) != napi_ok) return -1;
    *p = (const uint8_t *)data;
    return 0;
  }
  return -1;
}

static napi_value throw_code(napi_env env, int code) {
  /* the reference's JS engine errors keep their type and message (engine.ts:998 subarray of
     a missing dictionary chunk; Uint8Array.set out of range) */
  if (code == MIB_E_JS_TYPE_ERROR) napi_throw_type_error(env, NULL, "Cannot read property 'subarray' of undefined");
  else if (code == MIB_E_JS_RANGE_ERROR) napi_throw_range_error(env, NULL, "offset is out of bounds");
  else napi_throw_error(env, NULL, mib_strerror(code));
  return NULL;
}

static napi_value take(napi_env env, mib_buf *b) {
  napi_value out;
  void *dst;
  if (napi_create_buffer_copy(env, b->size, b->size ? (const void *)b->data : (const void *)"", &dst, &out) != napi_ok) {
    mib_buf_free(b);
    napi_throw_error(env, NULL, "brotli_amd: out of host memory");
    return NULL;
  }
  mib_buf_free(b);
  return out;
}

static int get_int(napi_env env, napi_value v, int dflt) {
  napi_valuetype t;
  int32_t r;
  if (napi_typeof(env, v, &t) != napi_ok || t != napi_number) return dflt;
  if (napi_get_value_int32(env, v, &r) != napi_ok) return dflt;
  return r;
}
static int64_t get_i64(napi_env env, napi_value v, int64_t dflt) {
  napi_valuetype t;
  int64_t r;
  if (napi_typeof(env, v, &t) != napi_ok || t != napi_number) return dflt;
  if (napi_get_value_int64(env, v, &r) != napi_ok) return dflt;
  return r;
}

/* encode(bytes, quality, lgwin, mode, dictionary|null) -> Buffer */
static napi_value js_encode(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  const uint8_t *p;
  size_t n;
  if (argc < 1 || get_bytes(env, argv[0], &p, &n)) {
    napi_throw_type_error(env, NULL, "input must be a Uint8Array");
    return NULL;
  }
  mib_enc_opts o;
  mib_enc_opts_default(&o);
  o.quality = get_int(env, argc > 1 ? argv[1] : NULL, o.quality);
  o.lgwin = get_int(env, argc > 2 ? argv[2] : NULL, o.lgwin);
  o.mode = get_int(env, argc > 3 ? argv[3] : NULL, o.mode);
  size_t dn = 0;
  if (argc > 4 && get_bytes(env, argv[4], &o.dict, &dn) == 0) o.dict_len = dn;
  else o.dict = NULL;
  mib_buf b = {0, 0};
  int rc = mib_encode(p, n, &o, &b);
  if (rc) return throw_code(env, rc);
  return take(env, &b);
}

/* decode(bytes, maxOutputSize|-1, exactSize|-1, dictionary|null) -> Buffer
 * throws Error("Brotli error code: N") or, for the size limit, an Error whose message
 * index.js rewrites; err.size carries the offending size. */
static napi_value js_decode(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  const uint8_t *p, *d = NULL;
  size_t n, dn = 0;
  if (argc < 1 || get_bytes(env, argv[0], &p, &n)) {
    napi_throw_type_error(env, NULL, "input must be a Uint8Array");
    return NULL;
  }
  int64_t max_out = argc > 1 ? get_i64(env, argv[1], -1) : -1;
  int64_t exact = argc > 2 ? get_i64(env, argv[2], -1) : -1;
  if (argc > 3 && get_bytes(env, argv[3], &d, &dn)) d = NULL;
  mib_buf b = {0, 0};
  int rc = mib_decode(p, n, d, d ? dn : 0, max_out, exact, &b);
  if (rc == MIB_E_OUTPUT_LIMIT) {
    napi_value err, msg, sz;
    napi_create_string_utf8(env, "Decompressed size exceeds limit", NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, NULL, msg, &err);
    napi_create_int64(env, (int64_t)b.size, &sz);
    napi_set_named_property(env, err, "size", sz);
    napi_throw(env, err);
    return NULL;
  }
  if (rc) return throw_code(env, rc);
  return take(env, &b);
}

static napi_value js_decoded_size(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], out;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  const uint8_t *p;
  size_t n;
  if (argc < 1 || get_bytes(env, argv[0], &p, &n)) {
    napi_throw_type_error(env, NULL, "input must be a Uint8Array");
    return NULL;
  }
  CHECK(env, napi_create_int64(env, mib_decoded_size(p, n), &out));
  return out;
}

static void encoder_finalize(napi_env env, void *data, void *hint) {
  (void)env;
  (void)hint;
  mib_encoder_free((mib_encoder *)data);
}

/* encoderNew(quality, lgwin, mode, dictionary|null, streamChunk) -> external handle (the
 * encoder copies the dictionary) */
static napi_value js_encoder_new(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5], out;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  mib_enc_opts o;
  mib_enc_opts_default(&o);
  o.quality = get_int(env, argc > 0 ? argv[0] : NULL, o.quality);
  o.lgwin = get_int(env, argc > 1 ? argv[1] : NULL, o.lgwin);
  o.mode = get_int(env, argc > 2 ? argv[2] : NULL, o.mode);
  size_t dn = 0;
  if (argc > 3 && get_bytes(env, argv[3], &o.dict, &dn) == 0) o.dict_len = dn;
  else o.dict = NULL;
  const int64_t sc = argc > 4 ? get_i64(env, argv[4], 0) : 0;
  o.stream_chunk = sc > 0 ? (uint64_t)sc : 0;
  mib_encoder *e = mib_encoder_new(&o);
  if (!e) return throw_code(env, MIB_E_OUT_OF_MEMORY);
  CHECK(env, napi_create_external(env, e, encoder_finalize, NULL, &out));
  return out;
}

static napi_value js_encoder_update(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  void *h;
  const uint8_t *p;
  size_t n;
  if (argc < 2 || napi_get_value_external(env, argv[0], &h) != napi_ok || get_bytes(env, argv[1], &p, &n)) {
    napi_throw_type_error(env, NULL, "update(chunk: Uint8Array)");
    return NULL;
  }
  mib_buf b = {0, 0};
  int rc = mib_encoder_update((mib_encoder *)h, p, n, &b);
  if (rc) return throw_code(env, rc);
  return take(env, &b);
}

static napi_value js_encoder_finish(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  void *h;
  if (argc < 1 || napi_get_value_external(env, argv[0], &h) != napi_ok) {
    napi_throw_type_error(env, NULL, "finish()");
    return NULL;
  }
  mib_buf b = {0, 0};
  int rc = mib_encoder_finish((mib_encoder *)h, &b);
  if (rc) return throw_code(env, rc);
  return take(env, &b);
}

/* encodeBatch([bytes...], quality, lgwin, mode, gpus, dictionary|null) -> [Buffer...]: one GPU
 * launch sequence (gpus >= 0: sharded over that many GPUs, 0 = all; -1 / absent: the default
 * device) */
static napi_value js_encode_batch(napi_env env, napi_callback_info info) {
  size_t argc = 6;
  napi_value argv[6], out;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  uint32_t k = 0;
  bool is_arr = false;
  if (argc < 1 || napi_is_array(env, argv[0], &is_arr) != napi_ok || !is_arr) {
    napi_throw_type_error(env, NULL, "encodeBatch(inputs: Uint8Array[])");
    return NULL;
  }
  CHECK(env, napi_get_array_length(env, argv[0], &k));
  mib_enc_opts o;
  mib_enc_opts_default(&o);
  o.quality = get_int(env, argc > 1 ? argv[1] : NULL, o.quality);
  o.lgwin = get_int(env, argc > 2 ? argv[2] : NULL, o.lgwin);
  o.mode = get_int(env, argc > 3 ? argv[3] : NULL, o.mode);
  size_t dn = 0;
  if (argc > 5 && get_bytes(env, argv[5], &o.dict, &dn) == 0) o.dict_len = dn;
  else o.dict = NULL;
  mib_span *in = (mib_span *)calloc(k ? k : 1, sizeof(mib_span));
  mib_buf *res = (mib_buf *)calloc(k ? k : 1, sizeof(mib_buf));
  int *st = (int *)calloc(k ? k : 1, sizeof(int));
  for (uint32_t i = 0; i < k; i++) {
    napi_value e;
    napi_get_element(env, argv[0], i, &e);
    if (get_bytes(env, e, &in[i].data, &in[i].size)) {
      free(in), free(res), free(st);
      napi_throw_type_error(env, NULL, "encodeBatch: every input must be a Uint8Array");
      return NULL;
    }
  }
  const int gpus = argc > 4 ? get_int(env, argv[4], -1) : -1;
  int rc = gpus >= 0 ? mib_encode_batch_n(in, k, &o, gpus, res, st) : mib_encode_batch(in, k, &o, res, st);
  free(in);
  if (rc) {
    free(res), free(st);
    return throw_code(env, rc);
  }
  napi_create_array_with_length(env, k, &out);
  for (uint32_t i = 0; i < k; i++) {
    napi_value v = take(env, &res[i]);
    if (!v) break;
    napi_set_element(env, out, i, v);
  }
  free(res);
  free(st);
  return out;
}

/* ---- asynchronous batches: the GPU work runs on a libuv worker thread (napi_async_work),
   the JS thread gets a Promise.  The inputs are COPIED into memory the addon owns before the
   work is queued: JS may transfer or detach an ArrayBuffer while the Promise is pending, and
   the worker must never read a buffer the JS heap has let go of. */
typedef struct {
  napi_async_work work;
  napi_deferred deferred;
  uint32_t k;
  int decode;       /* 0: encode batch, 1: decode batch */
  int gpus;         /* >= 0: sharded over that many GPUs (0 = all), else the default device */
  mib_enc_opts o;
  uint8_t *blob;    /* the inputs, back to back (owned) */
  uint8_t *dict;    /* encode: the customDictionary (owned copy), or NULL */
  mib_span *in;
  mib_buf *res;
  int *st;
  int rc;
} AsyncBatch;

static void async_free(AsyncBatch *a) {
  free(a->blob), free(a->dict), free(a->in), free(a->res), free(a->st), free(a);
}

static void async_execute(napi_env env, void *data) {
  AsyncBatch *a = (AsyncBatch *)data;
  if (a->gpus >= 0)
    a->rc = a->decode ? mib_decode_batch_n(a->in, a->k, a->gpus, a->res, a->st)
                      : mib_encode_batch_n(a->in, a->k, &a->o, a->gpus, a->res, a->st);
  else
    a->rc = a->decode ? mib_decode_batch(a->in, a->k, a->res, a->st) : mib_encode_batch(a->in, a->k, &a->o, a->res, a->st);
}

static void async_complete(napi_env env, napi_status status, void *data) {
  AsyncBatch *a = (AsyncBatch *)data;
  napi_value out, err;
  if (a->rc == 0 && status == napi_ok) {
    napi_create_array_with_length(env, a->k, &out);
    for (uint32_t i = 0; i < a->k; i++) {
      napi_value v;
      if (a->st[i]) {   /* a stream that failed to decode: its Error, in its slot */
        napi_value msg;
        napi_create_string_utf8(env, mib_strerror(a->st[i]), NAPI_AUTO_LENGTH, &msg);
        napi_create_error(env, NULL, msg, &v);
        mib_buf_free(&a->res[i]);
      } else {
        void *dst;
        napi_create_buffer_copy(env, a->res[i].size, a->res[i].size ? (const void *)a->res[i].data : (const void *)"", &dst, &v);
        mib_buf_free(&a->res[i]);
      }
      napi_set_element(env, out, i, v);
    }
    napi_resolve_deferred(env, a->deferred, out);
  } else {
    napi_value msg;
    napi_create_string_utf8(env, mib_strerror(a->rc ? a->rc : MIB_E_NO_DEVICE), NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, NULL, msg, &err);
    napi_reject_deferred(env, a->deferred, err);
    for (uint32_t i = 0; i < a->k; i++) mib_buf_free(&a->res[i]);
  }
  napi_delete_async_work(env, a->work);
  async_free(a);
}

/* encodeBatchAsync(inputs, quality, lgwin, mode, gpus, dictionary|null) /
 * decodeBatchAsync(inputs, gpus) -> Promise */
static napi_value start_async(napi_env env, napi_callback_info info, int decode) {
  size_t argc = 6;
  napi_value argv[6], promise, name;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  bool is_arr = false;
  uint32_t k = 0;
  if (argc < 1 || napi_is_array(env, argv[0], &is_arr) != napi_ok || !is_arr) {
    napi_throw_type_error(env, NULL, "inputs: Uint8Array[]");
    return NULL;
  }
  CHECK(env, napi_get_array_length(env, argv[0], &k));
  AsyncBatch *a = (AsyncBatch *)calloc(1, sizeof(AsyncBatch));
  a->k = k;
  a->decode = decode;
  a->gpus = decode ? (argc > 1 ? get_int(env, argv[1], -1) : -1) : (argc > 4 ? get_int(env, argv[4], -1) : -1);
  mib_enc_opts_default(&a->o);
  if (!decode) {
    a->o.quality = get_int(env, argc > 1 ? argv[1] : NULL, a->o.quality);
    a->o.lgwin = get_int(env, argc > 2 ? argv[2] : NULL, a->o.lgwin);
    a->o.mode = get_int(env, argc > 3 ? argv[3] : NULL, a->o.mode);
    const uint8_t *d;
    size_t dn;
    if (argc > 5 && get_bytes(env, argv[5], &d, &dn) == 0 && dn) {   /* (copied: JS may detach it) */
      a->dict = (uint8_t *)malloc(dn);
      if (!a->dict) {
        free(a);
        return throw_code(env, MIB_E_OUT_OF_MEMORY);
      }
      memcpy(a->dict, d, dn);
      a->o.dict = a->dict;
      a->o.dict_len = dn;
    }
  }
  a->in = (mib_span *)calloc(k ? k : 1, sizeof(mib_span));
  a->res = (mib_buf *)calloc(k ? k : 1, sizeof(mib_buf));
  a->st = (int *)calloc(k ? k : 1, sizeof(int));
  if (!a->in || !a->res || !a->st) {
    async_free(a);
    return throw_code(env, MIB_E_OUT_OF_MEMORY);
  }
  size_t total = 0;
  for (int pass = 0; pass < 2; pass++) {   /* sizes, then the copies */
    size_t at = 0;
    for (uint32_t i = 0; i < k; i++) {
      napi_value e;
      const uint8_t *p;
      size_t n;
      napi_get_element(env, argv[0], i, &e);
      if (get_bytes(env, e, &p, &n)) {
        async_free(a);
        napi_throw_type_error(env, NULL, "every input must be a Uint8Array");
        return NULL;
      }
      if (pass) {
        if (n) memcpy(a->blob + at, p, n);
        a->in[i].data = a->blob + at;
        a->in[i].size = n;
      }
      at += n;
    }
    if (!pass) {
      total = at;
      a->blob = (uint8_t *)malloc(total ? total : 1);
      if (!a->blob) {
        async_free(a);
        return throw_code(env, MIB_E_OUT_OF_MEMORY);
      }
    }
  }
  CHECK(env, napi_create_promise(env, &a->deferred, &promise));
  napi_create_string_utf8(env, decode ? "brotli_amd.decodeBatch" : "brotli_amd.encodeBatch", NAPI_AUTO_LENGTH, &name);
  CHECK(env, napi_create_async_work(env, NULL, name, async_execute, async_complete, a, &a->work));
  CHECK(env, napi_queue_async_work(env, a->work));
  return promise;
}
/* woff2Glyf(ttf) / woff2Hmtx(ttf) -> Buffer: the WOFF2-transformed glyf / hmtx table computed on
 * the GPU (the FONT-mode input of encode for a WOFF2 writer, reference README.md:63); hmtx
 * gives null when no transform applies */
static napi_value js_woff2(napi_env env, napi_callback_info info, int hmtx) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  const uint8_t *p;
  size_t n;
  if (argc < 1 || get_bytes(env, argv[0], &p, &n)) {
    napi_throw_type_error(env, NULL, "input must be a Uint8Array");
    return NULL;
  }
  mib_buf b = {0, 0};
  const int rc = hmtx ? mib_woff2_transform_hmtx(p, n, &b) : mib_woff2_transform_glyf(p, n, &b);
  if (rc) return throw_code(env, rc);
  if (hmtx && !b.size) {
    napi_value nul;
    CHECK(env, napi_get_null(env, &nul));
    return nul;
  }
  return take(env, &b);
}
static napi_value js_woff2_glyf(napi_env env, napi_callback_info info) { return js_woff2(env, info, 0); }
static napi_value js_woff2_hmtx(napi_env env, napi_callback_info info) { return js_woff2(env, info, 1); }
static napi_value js_encode_batch_async(napi_env env, napi_callback_info info) { return start_async(env, info, 0); }
static napi_value js_decode_batch_async(napi_env env, napi_callback_info info) { return start_async(env, info, 1); }

static napi_value init(napi_env env, napi_value exports) {
  napi_property_descriptor props[] = {
      {"encode", 0, js_encode, 0, 0, 0, napi_default, 0},
      {"decode", 0, js_decode, 0, 0, 0, napi_default, 0},
      {"decodedSize", 0, js_decoded_size, 0, 0, 0, napi_default, 0},
      {"encoderNew", 0, js_encoder_new, 0, 0, 0, napi_default, 0},
      {"encoderUpdate", 0, js_encoder_update, 0, 0, 0, napi_default, 0},
      {"encoderFinish", 0, js_encoder_finish, 0, 0, 0, napi_default, 0},
      {"encodeBatch", 0, js_encode_batch, 0, 0, 0, napi_default, 0},
      {"encodeBatchAsync", 0, js_encode_batch_async, 0, 0, 0, napi_default, 0},
      {"decodeBatchAsync", 0, js_decode_batch_async, 0, 0, 0, napi_default, 0},
      {"woff2Glyf", 0, js_woff2_glyf, 0, 0, 0, napi_default, 0},
      {"woff2Hmtx", 0, js_woff2_hmtx, 0, 0, 0, napi_default, 0},
  };
  napi_define_properties(env, exports, sizeof(props) / sizeof(props[0]), props);
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
