/*
 * benor_napi.c -- N-API addon: the reference's JavaScript/TypeScript surface
 * over the C ABI (include/benor.h).  Loaded by ../js/index.js.
 *
 * Exports (all thin; validation and semantics live in libbenor):
 *   networkCreate(N, F, initialValues, faultyList) -> external handle
 *       launchNodes.ts:4-44 (throws Error("Arrays don't match") /
 *       Error("faultyList doesnt have F faulties") with the reference's text)
 *   networkStart(handle, seed:BigInt, kMax[, stopAfter]) -> Promise<void>
 *       consensus.ts:3-8 + node.ts:167-188; runs the round loop kernel on a
 *       libuv worker thread (napi_async_work), so the event loop stays free;
 *       stopAfter (array of N delivery counts, null/undefined = never): GET /stop
 *       requests landing mid-run, node.ts:191-194 (bo_consensus_start_sched)
 *   networkStartLive(handle, seed:BigInt, kMax)     consensus.ts:3-8 as the reference
 *       runs it: launches the event-level kernel and returns; GET /stop served
 *       while it runs lands in it (bo_consensus_start_live)
 *   networkWait(handle) -> Promise<void>            end of a live run (bo_consensus_wait)
 *   liveStopEvents(handle) -> Array<number|null>    where a live run applied each /stop
 *   networkStop(handle) / nodeStop(handle, i)       consensus.ts:10-15, node.ts:191-194
 *   getState(handle, i) -> {killed, x, decided, k}  node.ts:197-199 (at once: a snapshot
 *       of a live run in flight)
 *   networkCreateTyped(N, F, Int8Array, Uint8Array) -> handle   the same, values encoded in JS
 *   getStatesRaw(handle) -> {buf, events}          the same records as an ArrayBuffer (decoded in JS)
 *   getStates(handle) -> {states, events}          every node at once (bo_get_states):
 *       events = the deliveries a live run's snapshot reflects, null otherwise
 *   consensusPoll(handle) -> boolean               a live run is in flight (bo_consensus_poll)
 *   status(handle, i) -> 500 | 200                  node.ts:33-39
 *   runTrials(cfg) -> Promise<BigUint64Array>       batch histogram (bo_run_trials)
 */
#define NAPI_VERSION 8
#include <node_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "benor.h"

#define NAPI_CALL(env, call)                                              \
    do {                                                                  \
        if ((call) != napi_ok) {                                          \
            napi_throw_error((env), NULL, "N-API call failed: " #call);   \
            return NULL;                                                  \
        }                                                                 \
    } while (0)

static void throw_bo(napi_env env, int rc) {
    const char *msg = bo_last_error();
    if (rc == BO_ERR_ARRAYS_DONT_MATCH || rc == BO_ERR_FAULTY_COUNT) {
        napi_throw_error(env, NULL, msg);   /* the reference's Error(message) text */
        return;
    }
    char buf[512];
    snprintf(buf, sizeof buf, "libbenor error %d: %s", rc, msg);
    napi_throw_error(env, NULL, buf);
}

static void finalize_net(napi_env env, void *data, void *hint) {
    (void)env; (void)hint;
    bo_network_destroy((bo_network *)data);
}

static bo_network *get_net(napi_env env, napi_value v) {
    void *p = NULL;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
        napi_throw_type_error(env, NULL, "expected a network handle");
        return NULL;
    }
    return (bo_network *)p;
}

static uint32_t get_u32(napi_env env, napi_value v, int *ok) {
    uint32_t x = 0;
    double d = 0;
    if (napi_get_value_double(env, v, &d) != napi_ok || d < 0 || d > 4294967295.0 || d != (double)(uint32_t)d) {
        *ok = 0;
        return 0;
    }
    x = (uint32_t)d;
    return x;
}

/* Value = 0 | 1 | "?"  ->  0, 1, 2;  anything else -> -2 (rejected by libbenor) */
static int8_t encode_value(napi_env env, napi_value v) {
    napi_valuetype t;
    napi_typeof(env, v, &t);
    if (t == napi_number) {
        double d = 0;
        napi_get_value_double(env, v, &d);
        if (d == 0) return 0;
        if (d == 1) return 1;
        return -2;
    }
    if (t == napi_string) {
        char s[4] = {0};
        size_t n = 0;
        napi_get_value_string_utf8(env, v, s, sizeof s, &n);
        if (n == 1 && s[0] == '?') return 2;
    }
    return -2;
}

static int read_array(napi_env env, napi_value arr, uint32_t *len_out) {
    bool is = false;
    napi_is_array(env, arr, &is);
    if (!is) return 0;
    napi_get_array_length(env, arr, len_out);
    return 1;
}

static napi_value network_create(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc < 4) { napi_throw_type_error(env, NULL, "networkCreate(N, F, initialValues, faultyList)"); return NULL; }
    int ok = 1;
    uint32_t N = get_u32(env, argv[0], &ok), F = get_u32(env, argv[1], &ok);
    uint32_t ni = 0, nf = 0;
    if (!ok || !read_array(env, argv[2], &ni) || !read_array(env, argv[3], &nf)) {
        napi_throw_type_error(env, NULL, "networkCreate: bad arguments");
        return NULL;
    }
    int8_t *init = (int8_t *)calloc(ni + 1, 1);
    uint8_t *fl = (uint8_t *)calloc(nf + 1, 1);
    for (uint32_t i = 0; i < ni; ++i) {
        napi_value e;
        napi_get_element(env, argv[2], i, &e);
        init[i] = encode_value(env, e);
    }
    for (uint32_t i = 0; i < nf; ++i) {   /* launchNodes.ts:12 counts `el === true` */
        napi_value e;
        bool b = false;
        napi_valuetype t;
        napi_get_element(env, argv[3], i, &e);
        napi_typeof(env, e, &t);
        if (t == napi_boolean) napi_get_value_bool(env, e, &b);
        fl[i] = b ? 1 : 0;
    }
    bo_network *net = NULL;
    int rc = bo_network_create(N, F, init, ni, fl, nf, &net);
    free(init);
    free(fl);
    if (rc) { throw_bo(env, rc); return NULL; }
    napi_value ext;
    NAPI_CALL(env, napi_create_external(env, net, finalize_net, NULL, &ext));
    return ext;
}

/* networkCreate with the values already encoded by the JS wrapper (js/index.js
 * encodeValues: Int8Array 0 / 1 / 2 = "?" / -2 invalid, Uint8Array 1 = faulty):
 * the same bo_network_create, no per-element N-API calls. */
static int typed_bytes(napi_env env, napi_value v, napi_typedarray_type want, void **data, uint32_t *len) {
    bool is = false;
    napi_is_typedarray(env, v, &is);
    if (!is) return 0;
    napi_typedarray_type t;
    size_t n = 0, off = 0;
    napi_value ab;
    if (napi_get_typedarray_info(env, v, &t, &n, data, &ab, &off) != napi_ok || t != want) return 0;
    *len = (uint32_t)n;
    return 1;
}

static napi_value network_create_typed(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    int ok = argc == 4;
    uint32_t N = ok ? get_u32(env, argv[0], &ok) : 0, F = ok ? get_u32(env, argv[1], &ok) : 0;
    void *init = NULL, *fl = NULL;
    uint32_t ni = 0, nf = 0;
    if (!ok || !typed_bytes(env, argv[2], napi_int8_array, &init, &ni) ||
        !typed_bytes(env, argv[3], napi_uint8_array, &fl, &nf)) {
        napi_throw_type_error(env, NULL, "networkCreateTyped(N, F, Int8Array, Uint8Array)");
        return NULL;
    }
    static const uint8_t none = 0;
    bo_network *net = NULL;
    int rc = bo_network_create(N, F, ni ? (const int8_t *)init : (const int8_t *)&none, ni,
                               nf ? (const uint8_t *)fl : &none, nf, &net);
    if (rc) { throw_bo(env, rc); return NULL; }
    napi_value ext;
    NAPI_CALL(env, napi_create_external(env, net, finalize_net, NULL, &ext));
    return ext;
}

/* ---- async start ---- */
typedef struct {
    napi_async_work work;
    napi_deferred deferred;
    napi_ref net_ref;
    bo_network *net;
    uint64_t seed;
    uint32_t k_max;
    uint32_t *stop_after;      /* [n_stop] or NULL */
    uint32_t n_stop;
    int rc;
    char err[512];
} start_job;

static void start_execute(napi_env env, void *data) {
    (void)env;
    start_job *j = (start_job *)data;
    j->rc = bo_consensus_start_sched(j->net, j->seed, j->k_max, j->stop_after, j->n_stop);
    if (j->rc) snprintf(j->err, sizeof j->err, "libbenor error %d: %s", j->rc, bo_last_error());
}

static void start_complete(napi_env env, napi_status status, void *data) {
    start_job *j = (start_job *)data;
    if (status == napi_ok && j->rc == 0) {
        napi_value u;
        napi_get_undefined(env, &u);
        napi_resolve_deferred(env, j->deferred, u);
    } else {
        napi_value msg, err;
        napi_create_string_utf8(env, j->rc ? j->err : "async work failed", NAPI_AUTO_LENGTH, &msg);
        napi_create_error(env, NULL, msg, &err);
        napi_reject_deferred(env, j->deferred, err);
    }
    napi_delete_reference(env, j->net_ref);
    napi_delete_async_work(env, j->work);
    free(j->stop_after);
    free(j);
}

static napi_value network_start(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc < 3) { napi_throw_type_error(env, NULL, "networkStart(handle, seed, kMax[, stopAfter])"); return NULL; }
    bo_network *net = get_net(env, argv[0]);
    if (!net) return NULL;
    start_job *j = (start_job *)calloc(1, sizeof *j);
    bool lossless = true;
    if (napi_get_value_bigint_uint64(env, argv[1], &j->seed, &lossless) != napi_ok) {
        double d = 0;
        napi_get_value_double(env, argv[1], &d);
        j->seed = (uint64_t)d;
    }
    int ok = 1;
    j->k_max = get_u32(env, argv[2], &ok);
    bool is_arr = false;
    if (argc > 3) napi_is_array(env, argv[3], &is_arr);
    if (is_arr) {                               /* stop schedule: one entry per node */
        uint32_t n = 0;
        napi_get_array_length(env, argv[3], &n);
        j->n_stop = n;
        j->stop_after = (uint32_t *)malloc(sizeof(uint32_t) * (n ? n : 1));
        for (uint32_t i = 0; i < n; ++i) {
            napi_value e;
            napi_valuetype t;
            napi_get_element(env, argv[3], i, &e);
            napi_typeof(env, e, &t);
            j->stop_after[i] = (t == napi_null || t == napi_undefined) ? 0xFFFFFFFFu : get_u32(env, e, &ok);
        }
    }
    if (!ok) {                                  /* kMax or a stopAfter entry is not a uint32 */
        free(j->stop_after);
        free(j);
        napi_throw_type_error(env, NULL, "kMax and stopAfter entries must be uint32 (stopAfter entries may be null)");
        return NULL;
    }
    j->net = net;
    napi_create_reference(env, argv[0], 1, &j->net_ref);   /* keep the handle alive while running */
    napi_value promise, name;
    NAPI_CALL(env, napi_create_promise(env, &j->deferred, &promise));
    NAPI_CALL(env, napi_create_string_utf8(env, "benor.start", NAPI_AUTO_LENGTH, &name));
    NAPI_CALL(env, napi_create_async_work(env, NULL, name, start_execute, start_complete, j, &j->work));
    NAPI_CALL(env, napi_queue_async_work(env, j->work));
    return promise;
}

static int get_seed(napi_env env, napi_value v, uint64_t *seed) {
    bool lossless = true;
    if (napi_get_value_bigint_uint64(env, v, seed, &lossless) == napi_ok) return 1;
    double d = 0;
    if (napi_get_value_double(env, v, &d) != napi_ok || d < 0) return 0;
    *seed = (uint64_t)d;
    return 1;
}

static napi_value network_start_live(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc < 3) { napi_throw_type_error(env, NULL, "networkStartLive(handle, seed, kMax)"); return NULL; }
    bo_network *net = get_net(env, argv[0]);
    if (!net) return NULL;
    uint64_t seed = 0;
    int ok = get_seed(env, argv[1], &seed);
    uint32_t k_max = get_u32(env, argv[2], &ok);
    if (!ok) { napi_throw_type_error(env, NULL, "seed must be a BigInt or number, kMax a uint32"); return NULL; }
    int rc = bo_consensus_start_live(net, seed, k_max);
    if (rc) { throw_bo(env, rc); return NULL; }
    return NULL;
}

/* ---- async wait for a live run ---- */
typedef struct {
    napi_async_work work;
    napi_deferred deferred;
    napi_ref net_ref;
    bo_network *net;
    int rc;
    char err[512];
} wait_job;

static void wait_execute(napi_env env, void *data) {
    (void)env;
    wait_job *j = (wait_job *)data;
    j->rc = bo_consensus_wait(j->net);
    if (j->rc) snprintf(j->err, sizeof j->err, "libbenor error %d: %s", j->rc, bo_last_error());
}

static void wait_complete(napi_env env, napi_status status, void *data) {
    wait_job *j = (wait_job *)data;
    if (status == napi_ok && j->rc == 0) {
        napi_value u;
        napi_get_undefined(env, &u);
        napi_resolve_deferred(env, j->deferred, u);
    } else {
        napi_value msg, err;
        napi_create_string_utf8(env, j->rc ? j->err : "async work failed", NAPI_AUTO_LENGTH, &msg);
        napi_create_error(env, NULL, msg, &err);
        napi_reject_deferred(env, j->deferred, err);
    }
    napi_delete_reference(env, j->net_ref);
    napi_delete_async_work(env, j->work);
    free(j);
}

static napi_value network_wait(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    bo_network *net = get_net(env, argv[0]);
    if (!net) return NULL;
    wait_job *j = (wait_job *)calloc(1, sizeof *j);
    j->net = net;
    napi_create_reference(env, argv[0], 1, &j->net_ref);
    napi_value promise, name;
    NAPI_CALL(env, napi_create_promise(env, &j->deferred, &promise));
    NAPI_CALL(env, napi_create_string_utf8(env, "benor.wait", NAPI_AUTO_LENGTH, &name));
    NAPI_CALL(env, napi_create_async_work(env, NULL, name, wait_execute, wait_complete, j, &j->work));
    NAPI_CALL(env, napi_queue_async_work(env, j->work));
    return promise;
}

static napi_value live_stop_events(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    bo_network *net = get_net(env, argv[0]);
    if (!net) return NULL;
    const uint32_t N = bo_network_size(net);
    uint32_t *ev = (uint32_t *)malloc(sizeof(uint32_t) * (N ? N : 1));
    int rc = bo_live_stop_events(net, ev, N);
    if (rc) { free(ev); throw_bo(env, rc); return NULL; }
    napi_value arr, v;
    napi_create_array_with_length(env, N, &arr);
    for (uint32_t i = 0; i < N; ++i) {
        if (ev[i] == 0xFFFFFFFFu) napi_get_null(env, &v);
        else napi_create_uint32(env, ev[i], &v);
        napi_set_element(env, arr, i, v);
    }
    free(ev);
    return arr;
}

static napi_value network_stop(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    bo_network *net = get_net(env, argv[0]);
    if (!net) return NULL;
    int rc = bo_consensus_stop(net);
    if (rc) { throw_bo(env, rc); return NULL; }
    return NULL;
}

static napi_value node_stop(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    bo_network *net = get_net(env, argv[0]);
    if (!net) return NULL;
    int ok = 1;
    uint32_t i = get_u32(env, argv[1], &ok);
    if (!ok) { napi_throw_type_error(env, NULL, "node index must be a uint32"); return NULL; }
    int rc = bo_node_stop(net, i);
    if (rc) { throw_bo(env, rc); return NULL; }
    return NULL;
}

static napi_value state_object(napi_env env, bo_node_state s) {
    napi_value o, v;
    NAPI_CALL(env, napi_create_object(env, &o));
    napi_get_boolean(env, s.killed != 0, &v);
    napi_set_named_property(env, o, "killed", v);
    if (s.x < 0) napi_get_null(env, &v);
    else if (s.x == 2) napi_create_string_utf8(env, "?", 1, &v);
    else napi_create_int32(env, s.x, &v);
    napi_set_named_property(env, o, "x", v);
    if (s.decided < 0) napi_get_null(env, &v);
    else napi_get_boolean(env, s.decided != 0, &v);
    napi_set_named_property(env, o, "decided", v);
    if (s.k < 0) napi_get_null(env, &v);
    else napi_create_int32(env, s.k, &v);
    napi_set_named_property(env, o, "k", v);
    return o;
}

static napi_value get_state(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    bo_network *net = get_net(env, argv[0]);
    if (!net) return NULL;
    int ok = 1;
    uint32_t i = get_u32(env, argv[1], &ok);
    if (!ok) { napi_throw_type_error(env, NULL, "node index must be a uint32"); return NULL; }
    bo_node_state s;
    int rc = bo_get_state(net, i, &s);
    if (rc) { throw_bo(env, rc); return NULL; }
    return state_object(env, s);
}

static napi_value get_states(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    bo_network *net = get_net(env, argv[0]);
    if (!net) return NULL;
    const uint32_t N = bo_network_size(net);
    bo_node_state *st = (bo_node_state *)malloc(sizeof(bo_node_state) * (N ? N : 1));
    uint64_t ev = 0;
    int rc = bo_get_states(net, st, N, &ev);
    if (rc) { free(st); throw_bo(env, rc); return NULL; }
    napi_value o, arr, v;
    napi_create_object(env, &o);
    napi_create_array_with_length(env, N, &arr);
    for (uint32_t i = 0; i < N; ++i) napi_set_element(env, arr, i, state_object(env, st[i]));
    free(st);
    napi_set_named_property(env, o, "states", arr);
    if (ev == UINT64_MAX) napi_get_null(env, &v);
    else napi_create_double(env, (double)ev, &v);
    napi_set_named_property(env, o, "events", v);
    return o;
}

/* getStates as raw bo_node_state records (8 bytes each: int8 killed, x,
 * decided, pad; int32 k) in an ArrayBuffer, decoded by js/index.js: one N-API
 * allocation instead of five calls per node. */
static napi_value get_states_raw(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    bo_network *net = get_net(env, argv[0]);
    if (!net) return NULL;
    const uint32_t N = bo_network_size(net);
    void *data = NULL;
    napi_value ab, o, v;
    NAPI_CALL(env, napi_create_arraybuffer(env, sizeof(bo_node_state) * (N ? N : 1), &data, &ab));
    uint64_t ev = 0;
    int rc = bo_get_states(net, (bo_node_state *)data, N, &ev);
    if (rc) { throw_bo(env, rc); return NULL; }
    napi_create_object(env, &o);
    napi_set_named_property(env, o, "buf", ab);
    if (ev == UINT64_MAX) napi_get_null(env, &v);
    else napi_create_double(env, (double)ev, &v);
    napi_set_named_property(env, o, "events", v);
    return o;
}

static napi_value consensus_poll(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    bo_network *net = get_net(env, argv[0]);
    if (!net) return NULL;
    int running = 0;
    int rc = bo_consensus_poll(net, &running);
    if (rc) { throw_bo(env, rc); return NULL; }
    napi_value v;
    napi_get_boolean(env, running != 0, &v);
    return v;
}

static napi_value status(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    bo_network *net = get_net(env, argv[0]);
    if (!net) return NULL;
    int ok = 1;
    uint32_t i = get_u32(env, argv[1], &ok);
    if (!ok) { napi_throw_type_error(env, NULL, "node index must be a uint32"); return NULL; }
    int code = bo_status(net, i);
    if (code < 0) { throw_bo(env, -code); return NULL; }
    napi_value v;
    napi_create_int32(env, code, &v);
    return v;
}

/* ---- async batch ---- */
typedef struct {
    napi_async_work work;
    napi_deferred deferred;
    bo_trials_cfg cfg;
    uint8_t *faulty;
    int8_t *init;
    uint64_t trial_begin, trial_count;
    uint64_t *hist;
    uint32_t *crash;
    uint32_t hlen;
    int rc;
    char err[512];
} trials_job;

static void trials_execute(napi_env env, void *data) {
    (void)env;
    trials_job *j = (trials_job *)data;
    j->rc = bo_run_trials(&j->cfg, j->trial_begin, j->trial_count, j->hist);
    if (j->rc) snprintf(j->err, sizeof j->err, "libbenor error %d: %s", j->rc, bo_last_error());
}

static void trials_complete(napi_env env, napi_status status, void *data) {
    trials_job *j = (trials_job *)data;
    if (status == napi_ok && j->rc == 0) {
        napi_value ab, ta;
        void *buf = NULL;
        napi_create_arraybuffer(env, sizeof(uint64_t) * j->hlen, &buf, &ab);
        memcpy(buf, j->hist, sizeof(uint64_t) * j->hlen);
        napi_create_typedarray(env, napi_biguint64_array, j->hlen, ab, 0, &ta);
        napi_resolve_deferred(env, j->deferred, ta);
    } else {
        napi_value msg, err;
        napi_create_string_utf8(env, j->rc ? j->err : "async work failed", NAPI_AUTO_LENGTH, &msg);
        napi_create_error(env, NULL, msg, &err);
        napi_reject_deferred(env, j->deferred, err);
    }
    napi_delete_async_work(env, j->work);
    free(j->faulty);
    free(j->init);
    free(j->hist);
    free(j->crash);
    free(j);
}

static int prop_u32(napi_env env, napi_value o, const char *k, uint32_t def, uint32_t *out) {
    bool has = false;
    napi_has_named_property(env, o, k, &has);
    if (!has) { *out = def; return 1; }
    napi_value v;
    napi_get_named_property(env, o, k, &v);
    int ok = 1;
    *out = get_u32(env, v, &ok);
    return ok;
}

static uint64_t prop_u64(napi_env env, napi_value o, const char *k, uint64_t def) {
    bool has = false;
    napi_has_named_property(env, o, k, &has);
    if (!has) return def;
    napi_value v;
    napi_get_named_property(env, o, k, &v);
    uint64_t x = 0;
    bool lossless = true;
    if (napi_get_value_bigint_uint64(env, v, &x, &lossless) == napi_ok) return x;
    double d = 0;
    napi_get_value_double(env, v, &d);
    return (uint64_t)d;
}

static napi_value run_trials(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
    if (argc < 1) { napi_throw_type_error(env, NULL, "runTrials(cfg)"); return NULL; }
    napi_value o = argv[0];
    trials_job *j = (trials_job *)calloc(1, sizeof *j);
    uint32_t kmax = 64;
    prop_u32(env, o, "N", 0, &j->cfg.N);
    prop_u32(env, o, "F", 0, &j->cfg.F);
    prop_u32(env, o, "kMax", 64, &kmax);
    j->cfg.k_max = kmax;
    j->cfg.seed = prop_u64(env, o, "seed", 0);
    j->trial_begin = prop_u64(env, o, "trialBegin", 0);
    j->trial_count = prop_u64(env, o, "trialCount", 1);
    uint32_t mode = BO_MODE_LOCKSTEP;
    prop_u32(env, o, "mode", BO_MODE_LOCKSTEP, &mode);          /* 0 lockstep, 1 random delivery, 2 event */
    j->cfg.mode = mode;
    prop_u32(env, o, "crashCount", 0, &j->cfg.crash_count);
    prop_u32(env, o, "crashWindow", 0, &j->cfg.crash_window);
    const uint32_t N = j->cfg.N;
    j->faulty = (uint8_t *)calloc(N + 1, 1);
    j->init = (int8_t *)calloc(N + 1, 1);
    bool has = false;
    napi_value arr;
    napi_has_named_property(env, o, "faultyList", &has);
    if (has) {
        napi_get_named_property(env, o, "faultyList", &arr);
        uint32_t n = 0;
        if (read_array(env, arr, &n))
            for (uint32_t i = 0; i < n && i < N; ++i) {
                napi_value e;
                bool b = false;
                napi_get_element(env, arr, i, &e);
                napi_get_value_bool(env, e, &b);
                j->faulty[i] = b ? 1 : 0;
            }
    } else {
        for (uint32_t i = 0; i < N && i < j->cfg.F; ++i) j->faulty[i] = 1;   /* start.ts:7-18 placement */
    }
    napi_has_named_property(env, o, "initialValues", &has);
    j->cfg.init_mode = has ? BO_INIT_FIXED : BO_INIT_RANDOM;
    if (has) {
        napi_get_named_property(env, o, "initialValues", &arr);
        uint32_t n = 0;
        if (read_array(env, arr, &n))
            for (uint32_t i = 0; i < n && i < N; ++i) {
                napi_value e;
                napi_get_element(env, arr, i, &e);
                j->init[i] = encode_value(env, e);
            }
    }
    napi_has_named_property(env, o, "crashAt", &has);
    if (has) {                                                   /* EVENT mode /stop schedule */
        napi_get_named_property(env, o, "crashAt", &arr);
        uint32_t n = 0;
        if (read_array(env, arr, &n)) {
            j->crash = (uint32_t *)malloc(sizeof(uint32_t) * (N + 1));
            for (uint32_t i = 0; i < N; ++i) j->crash[i] = 0xFFFFFFFFu;
            for (uint32_t i = 0; i < n && i < N; ++i) {
                napi_value e;
                napi_valuetype t;
                napi_get_element(env, arr, i, &e);
                napi_typeof(env, e, &t);
                if (t == napi_number) {
                    double d = 0;
                    napi_get_value_double(env, e, &d);
                    if (d >= 0 && d < 4294967295.0) j->crash[i] = (uint32_t)d;
                }
            }
            j->cfg.crash_at = j->crash;
        }
    }
    j->cfg.faulty = j->faulty;
    j->cfg.init = j->init;
    j->hlen = bo_hist_len(kmax);
    j->hist = (uint64_t *)calloc(j->hlen, sizeof(uint64_t));
    napi_value promise, name;
    NAPI_CALL(env, napi_create_promise(env, &j->deferred, &promise));
    NAPI_CALL(env, napi_create_string_utf8(env, "benor.runTrials", NAPI_AUTO_LENGTH, &name));
    NAPI_CALL(env, napi_create_async_work(env, NULL, name, trials_execute, trials_complete, j, &j->work));
    NAPI_CALL(env, napi_queue_async_work(env, j->work));
    return promise;
}

static napi_value init_module(napi_env env, napi_value exports) {
    napi_property_descriptor d[] = {
        {"networkCreate", NULL, network_create, NULL, NULL, NULL, napi_default, NULL},
        {"networkStart", NULL, network_start, NULL, NULL, NULL, napi_default, NULL},
        {"networkStartLive", NULL, network_start_live, NULL, NULL, NULL, napi_default, NULL},
        {"networkWait", NULL, network_wait, NULL, NULL, NULL, napi_default, NULL},
        {"liveStopEvents", NULL, live_stop_events, NULL, NULL, NULL, napi_default, NULL},
        {"networkStop", NULL, network_stop, NULL, NULL, NULL, napi_default, NULL},
        {"nodeStop", NULL, node_stop, NULL, NULL, NULL, napi_default, NULL},
        {"getState", NULL, get_state, NULL, NULL, NULL, napi_default, NULL},
        {"getStates", NULL, get_states, NULL, NULL, NULL, napi_default, NULL},
        {"getStatesRaw", NULL, get_states_raw, NULL, NULL, NULL, napi_default, NULL},
        {"networkCreateTyped", NULL, network_create_typed, NULL, NULL, NULL, napi_default, NULL},
        {"consensusPoll", NULL, consensus_poll, NULL, NULL, NULL, napi_default, NULL},
        {"status", NULL, status, NULL, NULL, NULL, napi_default, NULL},
        {"runTrials", NULL, run_trials, NULL, NULL, NULL, napi_default, NULL},
    };
    napi_define_properties(env, exports, sizeof d / sizeof d[0], d);
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init_module)
