/*
 * N-API addon over the libzkp_amd C ABI (include/zkp_amd.h).  This is the thin
 * binding a Node/TypeScript host (snarkjs' callers: reference app/src/helpers/zkp.ts:94,
 * dizkus-scripts/5_gen_proof.sh:8) uses in place of snarkjs.groth16.prove.
 *
 *   loadProver(zkeyPathOrBuffer, devices?)       -> external handle (zkey resident in HBM)
 *   prove(handle, wtnsBuffer, r32?, s32?)        -> Promise<{piA:[x,y], piB:[[x0,x1],[y0,y1]], piC:[x,y],
 *                                                            publicSignals:[...]}> (decimal strings)
 *   proveBatch(handle, [wtnsBuffer...], rs?, ss?) -> Promise<[result | Error, ...]> (zkp_prove_batch_status:
 *                                                    every proof attempted, per-proof errors)
 *   freeProver(handle)
 *   zkeyNew(r1csBuffer, ptauBuffer, device?)     -> Buffer (`snarkjs zkey new`, synchronous)
 *   zkeyBeacon(zkeyBuffer, beaconBuffer, numIterationsExp, device?, name?) -> Buffer (`zkey beacon`)
 *   zkeyContribute(zkeyBuffer, entropy, name?, device?) -> Buffer (`zkey contribute`)
 *   version()
 * prove()/proveBatch() run on the libuv threadpool (napi_async_work), so the JS main
 * thread is never blocked — the same async contract as snarkjs' Promise API.
 *
 * Handle lifetime: a job holds a reference on the handle object (no GC finalize while it
 * runs) and counts itself in the handle's in-flight counter; freeProver() on a handle with
 * jobs in flight only marks it, and the last job to finish frees the prover.  All of this
 * runs on the JS main thread (async work complete callbacks included), so no atomics.
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

typedef struct {
  zkp_prover* p;
  int inflight;  /* async jobs running on this handle */
  int freed;     /* freeProver() called: free when inflight drops to 0 */
} Slot;

static void slot_release_if_idle(Slot* slot) {
  if (slot->freed && slot->inflight == 0 && slot->p) {
    zkp_prover_free(slot->p);
    slot->p = NULL;
  }
}

static void finalize_prover(napi_env env, void* data, void* hint) {
  (void)env, (void)hint;
  /* explicit freeProver() is the normal path; GC of a live handle frees it too (a job in
   * flight holds a reference on the handle, so this never runs under one) */
  Slot* slot = (Slot*)data;
  if (slot->p) zkp_prover_free(slot->p);
  free(slot);
}

/* the live slot of a handle argument, or NULL (not a handle / already freed) */
static Slot* get_slot(napi_env env, napi_value v) {
  Slot* slot = NULL;
  if (napi_get_value_external(env, v, (void**)&slot) != napi_ok || !slot || !slot->p || slot->freed) return NULL;
  return slot;
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

/* zkeyNew(r1csBuffer, ptauBuffer, device?) -> Buffer: `snarkjs zkey new` (zkp_zkey_new),
 * synchronous -- a setup step, not a serving path */
static napi_value js_zkey_new(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  bool b0 = false, b1 = false;
  if (argc >= 2) {
    napi_is_buffer(env, argv[0], &b0);
    napi_is_buffer(env, argv[1], &b1);
  }
  if (!b0 || !b1) {
    napi_throw_type_error(env, NULL, "zkeyNew(r1csBuffer, ptauBuffer, device?)");
    return NULL;
  }
  int device = 0;
  if (argc > 2) napi_get_value_int32(env, argv[2], &device);
  void *r1cs, *ptau;
  size_t r1cs_len, ptau_len;
  NAPI_CALL(env, napi_get_buffer_info(env, argv[0], &r1cs, &r1cs_len));
  NAPI_CALL(env, napi_get_buffer_info(env, argv[1], &ptau, &ptau_len));
  uint8_t* out = NULL;
  size_t out_len = 0;
  zkp_status st = zkp_zkey_new(device, (const uint8_t*)r1cs, r1cs_len, (const uint8_t*)ptau, ptau_len, &out, &out_len);
  if (st != ZKP_OK) return throw_status(env, st);
  napi_value buf;
  void* dst = NULL;
  napi_status ns = napi_create_buffer(env, out_len, &dst, &buf);
  if (ns == napi_ok) memcpy(dst, out, out_len);
  zkp_buffer_free(out);
  if (ns != napi_ok) {
    napi_throw_error(env, NULL, "N-API call failed: napi_create_buffer");
    return NULL;
  }
  return buf;
}

/* a JS string argument into buf (NULL when absent / undefined / not a string) */
static const char* opt_string(napi_env env, napi_value v, char* buf, size_t cap) {
  napi_valuetype t;
  if (napi_typeof(env, v, &t) != napi_ok || t != napi_string) return NULL;
  size_t n = 0;
  if (napi_get_value_string_utf8(env, v, buf, cap, &n) != napi_ok) return NULL;
  return buf;
}

static napi_value buffer_out(napi_env env, uint8_t* out, size_t out_len) {
  napi_value buf;
  void* dst = NULL;
  napi_status ns = napi_create_buffer(env, out_len, &dst, &buf);
  if (ns == napi_ok) memcpy(dst, out, out_len);
  zkp_buffer_free(out);
  if (ns != napi_ok) {
    napi_throw_error(env, NULL, "N-API call failed: napi_create_buffer");
    return NULL;
  }
  return buf;
}

/* zkeyContribute(zkeyBuffer, entropyString, nameString?, device?) -> Buffer: `snarkjs zkey
 * contribute -e=... -n=...` (zkp_zkey_contribute_entropy: 64 bytes of /dev/urandom mixed with the
 * entropy, the contribution record appended), synchronous */
static napi_value js_zkey_contribute(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  bool b0 = false;
  char ent[4096], name[256];
  const char* e = NULL;
  if (argc >= 2) {
    napi_is_buffer(env, argv[0], &b0);
    e = opt_string(env, argv[1], ent, sizeof ent);
  }
  if (!b0 || !e) {
    napi_throw_type_error(env, NULL, "zkeyContribute(zkeyBuffer, entropyString, nameString?, device?)");
    return NULL;
  }
  const char* nm = argc > 2 ? opt_string(env, argv[2], name, sizeof name) : NULL;
  int device = 0;
  if (argc > 3) napi_get_value_int32(env, argv[3], &device);
  void* zkey;
  size_t zkey_len;
  NAPI_CALL(env, napi_get_buffer_info(env, argv[0], &zkey, &zkey_len));
  uint8_t* out = NULL;
  size_t out_len = 0;
  zkp_status st = zkp_zkey_contribute_entropy(device, (const uint8_t*)zkey, zkey_len, NULL, e, nm, &out, &out_len);
  if (st != ZKP_OK) return throw_status(env, st);
  return buffer_out(env, out, out_len);
}

/* zkeyBeacon(zkeyBuffer, beaconBuffer, numIterationsExp, device?, nameString?) -> Buffer:
 * `snarkjs zkey beacon` (zkp_zkey_beacon_named: GPU group arithmetic + the type-1 record),
 * synchronous */
static napi_value js_zkey_beacon(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  bool b0 = false, b1 = false;
  uint32_t e = 0;
  if (argc >= 3) {
    napi_is_buffer(env, argv[0], &b0);
    napi_is_buffer(env, argv[1], &b1);
  }
  if (!b0 || !b1 || napi_get_value_uint32(env, argv[2], &e) != napi_ok) {
    napi_throw_type_error(env, NULL, "zkeyBeacon(zkeyBuffer, beaconBuffer, numIterationsExp, device?)");
    return NULL;
  }
  int device = 0;
  if (argc > 3) napi_get_value_int32(env, argv[3], &device);
  void *zkey, *beacon;
  size_t zkey_len, beacon_len;
  NAPI_CALL(env, napi_get_buffer_info(env, argv[0], &zkey, &zkey_len));
  NAPI_CALL(env, napi_get_buffer_info(env, argv[1], &beacon, &beacon_len));
  uint8_t* out = NULL;
  size_t out_len = 0;
  char name[256];
  const char* nm = argc > 4 ? opt_string(env, argv[4], name, sizeof name) : NULL;
  zkp_status st = zkp_zkey_beacon_named(device, (const uint8_t*)zkey, zkey_len, (const uint8_t*)beacon, beacon_len, e,
                                        nm, &out, &out_len);
  if (st != ZKP_OK) return throw_status(env, st);
  return buffer_out(env, out, out_len);
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
  Slot* slot = (Slot*)calloc(1, sizeof *slot);
  slot->p = p;
  napi_value ext;
  NAPI_CALL(env, napi_create_external(env, slot, finalize_prover, NULL, &ext));
  return ext;
}

static napi_value js_free(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  Slot* slot = NULL;
  NAPI_CALL(env, napi_get_value_external(env, argv[0], (void**)&slot));
  if (slot) {
    slot->freed = 1;
    slot_release_if_idle(slot);  /* deferred to the last in-flight job otherwise */
  }
  return NULL;
}

typedef struct {
  napi_async_work work;
  napi_deferred deferred;
  napi_ref wtns_ref;
  napi_ref handle_ref;
  Slot* slot;
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
  j->slot->inflight--;
  slot_release_if_idle(j->slot);
  napi_delete_reference(env, j->handle_ref);
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
  Slot* slot = get_slot(env, argv[0]);
  if (!slot) {
    free(j);
    napi_throw_type_error(env, NULL, "invalid or freed prover handle");
    return NULL;
  }
  j->slot = slot;
  j->p = slot->p;
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
  napi_create_reference(env, argv[1], 1, &j->wtns_ref);   /* keep the Buffer alive while proving */
  napi_create_reference(env, argv[0], 1, &j->handle_ref); /* ... and the handle (no finalize) */
  slot->inflight++;
  napi_value promise, name;
  NAPI_CALL(env, napi_create_promise(env, &j->deferred, &promise));
  NAPI_CALL(env, napi_create_string_utf8(env, "zkp_prove", NAPI_AUTO_LENGTH, &name));
  NAPI_CALL(env, napi_create_async_work(env, NULL, name, prove_exec, prove_done, j, &j->work));
  NAPI_CALL(env, napi_queue_async_work(env, j->work));
  return promise;
}

/* ---- proveBatch: zkp_prove_batch_status over an array of witness Buffers */
typedef struct {
  napi_async_work work;
  napi_deferred deferred;
  napi_ref arr_ref, handle_ref;
  Slot* slot;
  zkp_prover* p;
  int n;
  const uint8_t** wtns;
  size_t* lens;
  uint8_t *rbuf, *sbuf;            /* n x 32 bytes each, or NULL */
  const uint8_t **rptr, **sptr;
  zkp_proof* proofs;
  uint8_t* pub;                    /* n x npub x 32 */
  zkp_status* st;
  zkp_status rc;
  char err[512];
} BatchJob;

static void batch_free(BatchJob* j) {
  free(j->wtns), free(j->lens), free(j->rbuf), free(j->sbuf), free(j->rptr), free(j->sptr);
  free(j->proofs), free(j->pub), free(j->st);
  free(j);
}

static void batch_exec(napi_env env, void* data) {
  (void)env;
  BatchJob* j = (BatchJob*)data;
  j->rc = zkp_prove_batch_status(j->p, j->wtns, j->lens, j->n, (const uint8_t* const*)j->rptr,
                                 (const uint8_t* const*)j->sptr, j->proofs, j->st);
  if (j->rc != ZKP_OK) snprintf(j->err, sizeof j->err, "%s", zkp_last_error());
}

static napi_value proof_object(napi_env env, const zkp_proof* pr, const uint8_t* pub) {
  napi_value res, pb, pa;
  napi_create_object(env, &res);
  napi_set_named_property(env, res, "piA", pair(env, pr->pi_a[0], pr->pi_a[1]));
  napi_create_array_with_length(env, 2, &pb);
  napi_set_element(env, pb, 0, pair(env, pr->pi_b[0][0], pr->pi_b[0][1]));
  napi_set_element(env, pb, 1, pair(env, pr->pi_b[1][0], pr->pi_b[1][1]));
  napi_set_named_property(env, res, "piB", pb);
  napi_set_named_property(env, res, "piC", pair(env, pr->pi_c[0], pr->pi_c[1]));
  napi_create_array_with_length(env, pr->n_public, &pa);
  for (uint32_t i = 0; i < pr->n_public && i < pr->public_capacity; ++i)
    napi_set_element(env, pa, i, dec_str(env, pub + 32 * (size_t)i));
  napi_set_named_property(env, res, "publicSignals", pa);
  return res;
}

static void batch_done(napi_env env, napi_status status, void* data) {
  BatchJob* j = (BatchJob*)data;
  (void)status;
  napi_value arr;
  napi_create_array_with_length(env, (size_t)j->n, &arr);
  for (int i = 0; i < j->n; ++i) {
    napi_value v;
    if (j->st[i] == ZKP_OK) {
      v = proof_object(env, &j->proofs[i], j->proofs[i].public_signals);
    } else {
      napi_value msg, code;
      char c[16], m[96];
      snprintf(c, sizeof c, "%d", (int)j->st[i]);
      snprintf(m, sizeof m, "proof %d failed with status %d", i, (int)j->st[i]);
      napi_create_string_utf8(env, j->rc != ZKP_OK && j->n == 1 ? j->err : m, NAPI_AUTO_LENGTH, &msg);
      napi_create_string_utf8(env, c, NAPI_AUTO_LENGTH, &code);
      napi_create_error(env, code, msg, &v);
    }
    napi_set_element(env, arr, (uint32_t)i, v);
  }
  napi_resolve_deferred(env, j->deferred, arr);
  napi_delete_reference(env, j->arr_ref);
  j->slot->inflight--;
  slot_release_if_idle(j->slot);
  napi_delete_reference(env, j->handle_ref);
  napi_delete_async_work(env, j->work);
  batch_free(j);
}

/* rs / ss: undefined or an array of n 32-byte Buffers */
static int get_scalars(napi_env env, napi_value v, int n, uint8_t** buf, const uint8_t*** ptr) {
  napi_valuetype t;
  napi_typeof(env, v, &t);
  if (t == napi_undefined || t == napi_null) return 0;
  bool is_arr = false;
  napi_is_array(env, v, &is_arr);
  uint32_t len = 0;
  if (!is_arr || napi_get_array_length(env, v, &len) != napi_ok || (int)len != n) return -1;
  *buf = (uint8_t*)calloc((size_t)n + 1, 32);
  *ptr = (const uint8_t**)calloc((size_t)n + 1, sizeof **ptr);
  for (int i = 0; i < n; ++i) {
    napi_value e;
    napi_get_element(env, v, (uint32_t)i, &e);
    if (get_scalar(env, e, *buf + 32 * (size_t)i) != 1) return -1;
    (*ptr)[i] = *buf + 32 * (size_t)i;
  }
  return 1;
}

static napi_value js_prove_batch(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 2) {
    napi_throw_type_error(env, NULL, "proveBatch(handle, [wtnsBuffer...], rs?, ss?)");
    return NULL;
  }
  Slot* slot = get_slot(env, argv[0]);
  if (!slot) {
    napi_throw_type_error(env, NULL, "invalid or freed prover handle");
    return NULL;
  }
  bool is_arr = false;
  uint32_t n = 0;
  napi_is_array(env, argv[1], &is_arr);
  if (!is_arr || napi_get_array_length(env, argv[1], &n) != napi_ok) {
    napi_throw_type_error(env, NULL, "witnesses must be an array of Buffers");
    return NULL;
  }
  BatchJob* j = (BatchJob*)calloc(1, sizeof *j);
  j->slot = slot;
  j->p = slot->p;
  j->n = (int)n;
  j->wtns = (const uint8_t**)calloc((size_t)n + 1, sizeof *j->wtns);
  j->lens = (size_t*)calloc((size_t)n + 1, sizeof *j->lens);
  for (uint32_t i = 0; i < n; ++i) {
    napi_value e;
    void* d;
    napi_get_element(env, argv[1], i, &e);
    if (napi_get_buffer_info(env, e, &d, &j->lens[i]) != napi_ok) {
      batch_free(j);
      napi_throw_type_error(env, NULL, "witnesses must be an array of Buffers");
      return NULL;
    }
    j->wtns[i] = (const uint8_t*)d;
  }
  if ((argc > 2 && get_scalars(env, argv[2], (int)n, &j->rbuf, &j->rptr) < 0) ||
      (argc > 3 && get_scalars(env, argv[3], (int)n, &j->sbuf, &j->sptr) < 0)) {
    batch_free(j);
    napi_throw_type_error(env, NULL, "rs/ss must be arrays of n 32-byte Buffers");
    return NULL;
  }
  uint32_t nv, npub, dom;
  zkp_prover_info(j->p, &nv, &npub, &dom);
  j->proofs = (zkp_proof*)calloc((size_t)n + 1, sizeof *j->proofs);
  j->pub = (uint8_t*)calloc(((size_t)n + 1) * ((size_t)npub + 1), 32);
  j->st = (zkp_status*)calloc((size_t)n + 1, sizeof *j->st);
  for (uint32_t i = 0; i < n; ++i) {
    j->proofs[i].public_capacity = npub;
    j->proofs[i].public_signals = j->pub + (size_t)i * ((size_t)npub + 1) * 32;
  }
  napi_create_reference(env, argv[1], 1, &j->arr_ref);     /* the array keeps every Buffer alive */
  napi_create_reference(env, argv[0], 1, &j->handle_ref);
  slot->inflight++;
  napi_value promise, name;
  NAPI_CALL(env, napi_create_promise(env, &j->deferred, &promise));
  NAPI_CALL(env, napi_create_string_utf8(env, "zkp_prove_batch", NAPI_AUTO_LENGTH, &name));
  NAPI_CALL(env, napi_create_async_work(env, NULL, name, batch_exec, batch_done, j, &j->work));
  NAPI_CALL(env, napi_queue_async_work(env, j->work));
  return promise;
}

static napi_value init(napi_env env, napi_value exports) {
  napi_property_descriptor props[] = {
      {"version", NULL, js_version, NULL, NULL, NULL, napi_default, NULL},
      {"loadProver", NULL, js_load, NULL, NULL, NULL, napi_default, NULL},
      {"prove", NULL, js_prove, NULL, NULL, NULL, napi_default, NULL},
      {"proveBatch", NULL, js_prove_batch, NULL, NULL, NULL, napi_default, NULL},
      {"freeProver", NULL, js_free, NULL, NULL, NULL, napi_default, NULL},
      {"zkeyNew", NULL, js_zkey_new, NULL, NULL, NULL, napi_default, NULL},
      {"zkeyBeacon", NULL, js_zkey_beacon, NULL, NULL, NULL, napi_default, NULL},
      {"zkeyContribute", NULL, js_zkey_contribute, NULL, NULL, NULL, napi_default, NULL},
  };
  napi_define_properties(env, exports, sizeof props / sizeof props[0], props);
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
