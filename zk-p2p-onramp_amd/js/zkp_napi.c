/*
 * N-API addon over the libzkp_amd C ABI (include/zkp_amd.h).  This is the thin
 * binding a Node/TypeScript host (snarkjs' callers: reference app/src/helpers/zkp.ts:94,
 * dizkus-scripts/5_gen_proof.sh:8) uses in place of snarkjs.groth16.prove.
 *
 *   loadProver(zkeyPathOrBuffer, devices?)       -> external handle (zkey resident in HBM)
 *   prove(handle, wtnsBuffer, r32?, s32?)        -> Promise<{piA:[x,y], piB:[[x0,x1],[y0,y1]], piC:[x,y],
 *                                                            publicSignals:[...]}> (decimal strings)
 *   freeProver(handle)
 *   version()
 * prove() runs zkp_prove on the libuv threadpool (napi_async_work), so the JS main
 * thread is never blocked — the same async contract as snarkjs' Promise API.
 */
#define NAPI_VERSION 8
#include <node_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/zkp_amd.h"

#define NAPI_CALL(env, call)                                   \
  do {                                                         \
    if ((call) != napi_ok) {                                   \
      napi_throw_error((env), NULL, "N-API call failed: " #call); \
      return NULL;                                             \
    }                                                          \
  } while (0)

static void finalize_prover(napi_env env, void* data, void* hint) {
  (void)env, (void)hint;
  /* explicit freeProver() is the normal path; GC of a live handle frees it too */
  zkp_prover** slot = (zkp_prover**)data;
  if (*slot) zkp_prover_free(*slot);
  free(slot);
}

static napi_value throw_status(napi_env env, zkp_status st) {
  char code[16];
  snprintf(code, sizeof code, "%d", (int)st);
  napi_throw_error(env, code, zkp_last_error());
  return NULL;
}

static napi_value js_version(napi_env env, napi_callback_info info) {
  (void)info;
  napi_value s;
  NAPI_CALL(env, napi_create_string_utf8(env, zkp_version(), NAPI_AUTO_LENGTH, &s));
  return s;
}

static napi_value js_load(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 1) {
    napi_throw_type_error(env, NULL, "loadProver(zkeyPathOrBuffer, devices?)");
    return NULL;
  }
  int devs[64];
  int ndev = 0;
  if (argc > 1) {
    bool is_arr = false;
    napi_is_array(env, argv[1], &is_arr);
    if (is_arr) {
      uint32_t len = 0;
      napi_get_array_length(env, argv[1], &len);
      for (uint32_t i = 0; i < len && i < 64; ++i) {
        napi_value v;
        napi_get_element(env, argv[1], i, &v);
        napi_get_value_int32(env, v, &devs[ndev++]);
      }
    }
  }
  zkp_prover* p = NULL;
  zkp_status st;
  bool is_buf = false;
  napi_is_buffer(env, argv[0], &is_buf);
  if (is_buf) {
    void* data;
    size_t len;
    NAPI_CALL(env, napi_get_buffer_info(env, argv[0], &data, &len));
    st = zkp_prover_load_mem((const uint8_t*)data, len, ndev ? devs : NULL, ndev, &p);
  } else {
    char path[4096];
    size_t n;
    NAPI_CALL(env, napi_get_value_string_utf8(env, argv[0], path, sizeof path, &n));
    st = zkp_prover_load_file(path, ndev ? devs : NULL, ndev, &p);
  }
  if (st != ZKP_OK) return throw_status(env, st);
  zkp_prover** slot = (zkp_prover**)malloc(sizeof *slot);
  *slot = p;
  napi_value ext;
  NAPI_CALL(env, napi_create_external(env, slot, finalize_prover, NULL, &ext));
  return ext;
}

static napi_value js_free(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  zkp_prover** slot;
  NAPI_CALL(env, napi_get_value_external(env, argv[0], (void**)&slot));
  if (*slot) zkp_prover_free(*slot);
  *slot = NULL;
  return NULL;
}

typedef struct {
  napi_async_work work;
  napi_deferred deferred;
  napi_ref wtns_ref;
  zkp_prover* p;
  const uint8_t* wtns;
  size_t len;
  uint8_t r[32], s[32];
  int have_r, have_s;
  zkp_proof proof;
  uint8_t* pub;
  zkp_status st;
  char err[512];
} ProveJob;

static void prove_exec(napi_env env, void* data) {
  (void)env;
  ProveJob* j = (ProveJob*)data;
  j->st = zkp_prove(j->p, j->wtns, j->len, j->have_r ? j->r : NULL, j->have_s ? j->s : NULL, &j->proof);
  if (j->st != ZKP_OK) snprintf(j->err, sizeof j->err, "%s", zkp_last_error());
}

/* 32-byte LE -> decimal string */
static void le_to_dec(const uint8_t* le, char* out) {
  uint32_t w[8];
  for (int i = 0; i < 8; ++i) w[i] = (uint32_t)le[4 * i] | (uint32_t)le[4 * i + 1] << 8 | (uint32_t)le[4 * i + 2] << 16 |
                                     (uint32_t)le[4 * i + 3] << 24;
  char tmp[96];
  int n = 0;
  for (;;) {
    int zero = 1;
    for (int i = 0; i < 8; ++i)
      if (w[i]) zero = 0;
    if (zero) break;
    uint64_t rem = 0;
    for (int i = 7; i >= 0; --i) {
      uint64_t cur = (rem << 32) | w[i];
      w[i] = (uint32_t)(cur / 10);
      rem = cur % 10;
    }
    tmp[n++] = (char)('0' + rem);
  }
  if (!n) tmp[n++] = '0';
  for (int i = 0; i < n; ++i) out[i] = tmp[n - 1 - i];
  out[n] = 0;
}

static napi_value dec_str(napi_env env, const uint8_t* le) {
  char buf[96];
  le_to_dec(le, buf);
  napi_value s;
  napi_create_string_utf8(env, buf, NAPI_AUTO_LENGTH, &s);
  return s;
}

static napi_value pair(napi_env env, const uint8_t* a, const uint8_t* b) {
  napi_value arr;
  napi_create_array_with_length(env, 2, &arr);
  napi_set_element(env, arr, 0, dec_str(env, a));
  napi_set_element(env, arr, 1, dec_str(env, b));
  return arr;
}

static void prove_done(napi_env env, napi_status status, void* data) {
  ProveJob* j = (ProveJob*)data;
  (void)status;
  if (j->st != ZKP_OK) {
    napi_value msg, code, err;
    char c[16];
    snprintf(c, sizeof c, "%d", (int)j->st);
    napi_create_string_utf8(env, j->err, NAPI_AUTO_LENGTH, &msg);
    napi_create_string_utf8(env, c, NAPI_AUTO_LENGTH, &code);
    napi_create_error(env, code, msg, &err);
    napi_reject_deferred(env, j->deferred, err);
  } else {
    napi_value res, pb, pub;
    napi_create_object(env, &res);
    napi_set_named_property(env, res, "piA", pair(env, j->proof.pi_a[0], j->proof.pi_a[1]));
    napi_create_array_with_length(env, 2, &pb);
    napi_set_element(env, pb, 0, pair(env, j->proof.pi_b[0][0], j->proof.pi_b[0][1]));
    napi_set_element(env, pb, 1, pair(env, j->proof.pi_b[1][0], j->proof.pi_b[1][1]));
    napi_set_named_property(env, res, "piB", pb);
    napi_set_named_property(env, res, "piC", pair(env, j->proof.pi_c[0], j->proof.pi_c[1]));
    napi_create_array_with_length(env, j->proof.n_public, &pub);
    for (uint32_t i = 0; i < j->proof.n_public && i < j->proof.public_capacity; ++i)
      napi_set_element(env, pub, i, dec_str(env, j->pub + 32 * (size_t)i));
    napi_set_named_property(env, res, "publicSignals", pub);
    napi_resolve_deferred(env, j->deferred, res);
  }
  napi_delete_reference(env, j->wtns_ref);
  napi_delete_async_work(env, j->work);
  free(j->pub);
  free(j);
}

static int get_scalar(napi_env env, napi_value v, uint8_t out[32]) {
  napi_valuetype t;
  napi_typeof(env, v, &t);
  if (t == napi_undefined || t == napi_null) return 0;
  bool is_buf = false;
  napi_is_buffer(env, v, &is_buf);
  if (!is_buf) return -1;
  void* d;
  size_t n;
  napi_get_buffer_info(env, v, &d, &n);
  if (n != 32) return -1;
  memcpy(out, d, 32);
  return 1;
}

static napi_value js_prove(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 2) {
    napi_throw_type_error(env, NULL, "prove(handle, wtnsBuffer, r32?, s32?)");
    return NULL;
  }
  ProveJob* j = (ProveJob*)calloc(1, sizeof *j);
  zkp_prover** slot;
  if (napi_get_value_external(env, argv[0], (void**)&slot) != napi_ok || !*slot) {
    free(j);
    napi_throw_type_error(env, NULL, "invalid or freed prover handle");
    return NULL;
  }
  j->p = *slot;
  void* data;
  if (napi_get_buffer_info(env, argv[1], &data, &j->len) != napi_ok) {
    free(j);
    napi_throw_type_error(env, NULL, "wtns must be a Buffer");
    return NULL;
  }
  j->wtns = (const uint8_t*)data;
  j->have_r = argc > 2 ? get_scalar(env, argv[2], j->r) : 0;
  j->have_s = argc > 3 ? get_scalar(env, argv[3], j->s) : 0;
  if (j->have_r < 0 || j->have_s < 0) {
    free(j);
    napi_throw_type_error(env, NULL, "r/s must be 32-byte Buffers");
    return NULL;
  }
  uint32_t nv, npub, dom;
  zkp_prover_info(j->p, &nv, &npub, &dom);
  j->pub = (uint8_t*)calloc((size_t)npub + 1, 32);
  j->proof.public_capacity = npub;
  j->proof.public_signals = j->pub;
  napi_create_reference(env, argv[1], 1, &j->wtns_ref);  /* keep the Buffer alive while proving */
  napi_value promise, name;
  NAPI_CALL(env, napi_create_promise(env, &j->deferred, &promise));
  NAPI_CALL(env, napi_create_string_utf8(env, "zkp_prove", NAPI_AUTO_LENGTH, &name));
  NAPI_CALL(env, napi_create_async_work(env, NULL, name, prove_exec, prove_done, j, &j->work));
  NAPI_CALL(env, napi_queue_async_work(env, j->work));
  return promise;
}

static napi_value init(napi_env env, napi_value exports) {
  napi_property_descriptor props[] = {
      {"version", NULL, js_version, NULL, NULL, NULL, napi_default, NULL},
      {"loadProver", NULL, js_load, NULL, NULL, NULL, napi_default, NULL},
      {"prove", NULL, js_prove, NULL, NULL, NULL, napi_default, NULL},
      {"freeProver", NULL, js_free, NULL, NULL, NULL, napi_default, NULL},
  };
  napi_define_properties(env, exports, sizeof props / sizeof props[0], props);
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
