/* Host-side helper of the N = 1 drop-in (FJSPSimulation.py facade), a CPython extension:
 *
 *  obs_dicts(i32, i8, f32, mask): one env's observation columns from the pinned step record ->
 *    the reference's dict of numpy arrays, built with the CPython / numpy C APIs in one call
 *    (spec.obs_dicts is the same function in Python, and the definition the tests compare this
 *    one with).  Reference dict layout: PickupStationAgent.py:87-96, AGVAgent.py:60-75,
 *    MachineAgent.py:64-69, PackagingAgent.py:266-271 — every field a 0-d array of its dtype
 *    (np.array(x, dtype=...)), the AGV's position a 2-vector, every action mask its own int8
 *    array (get_action_mask().astype).
 *
 *  stepper(...) / step(stepper, actions): FJSPSimulation.step's common case in one call — a
 *    dict of the eight agents in the canonical order with plain int actions 0..253 — the action
 *    bytes, the step server's request (fjsp_server_step_actions, called through the pointer the
 *    facade hands over, the GIL released while it waits) and the reference's return values
 *    (FJSPSimulation.py:144-242: observations, rewards, terminations, truncations, infos).  Any
 *    other dict returns None before any side effect and the facade takes its Python path.
 *
 * Inputs are the record's column views / addresses (pinned host memory the kernels write).  No
 * GPU code of its own. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#define NPY_NO_DEPRECATED_API NPY_1_7_API_VERSION
#include <numpy/arrayobject.h>
#include <string.h>

#define N_AG 8
#define N_PICK 7
#define N_AGV 12
static const char* AGENTS[N_AG] = {"pickup_station", "agv", "small_machine", "big_machine",
                                   "packaging_blue_1", "packaging_blue_2", "packaging_red", "packaging_green"};
static const char* PICK[N_PICK] = {"order_size", "products_remaining", "next_product_type", "next_product_color",
                                   "current_tray_type", "current_tray_color", "current_tray_count"};
static const char* AGV[N_AGV] = {"position", "carrying_tray", "tray_product_count", "tray_type",
                                 "tray_needs_processing", "tray_needs_packaging", "pickup_ready_trays",
                                 "small_machine_busy", "big_machine_busy", "small_machine_ready",
                                 "big_machine_ready", "storage_tray_count"};
static const int MASK_OFF[N_AG + 1] = {0, 3, 11, 14, 17, 20, 23, 26, 29};

static PyObject *s_agents[N_AG], *s_pick[N_PICK], *s_agv[N_AGV];
static PyObject *s_busy, *s_prog, *s_queue, *s_mask, *s_ares, *s_stime, *s_ocomp, *s_tpack;

static PyObject* scalar(int type, const void* v, size_t bytes) {
    PyObject* a = PyArray_SimpleNew(0, NULL, type);
    if (a) memcpy(PyArray_DATA((PyArrayObject*)a), v, bytes);
    return a;
}

static PyObject* vec(int type, npy_intp n, const void* v, size_t bytes) {
    PyObject* a = PyArray_SimpleNew(1, &n, type);
    if (a) memcpy(PyArray_DATA((PyArrayObject*)a), v, bytes);
    return a;
}

/* d[key] = value, stealing the value reference; 0 on success */
static int put(PyObject* d, PyObject* key, PyObject* v) {
    if (!v) return -1;
    const int r = PyDict_SetItem(d, key, v);
    Py_DECREF(v);
    return r;
}

static int get_buf(PyObject* o, Py_buffer* b, Py_ssize_t need, const char* what) {
    if (PyObject_GetBuffer(o, b, PyBUF_C_CONTIGUOUS) != 0) return -1;
    if (b->len < need) {
        PyBuffer_Release(b);
        PyErr_Format(PyExc_ValueError, "obs_dicts: %s holds %zd bytes, needs %zd", what, b->len, need);
        return -1;
    }
    return 0;
}

/* the reference's observation dict of one env from its record columns */
static PyObject* build_obs(const int32_t* a, const int8_t* b, const float* c, const int8_t* m) {
    PyObject* obs = PyDict_New();
    if (!obs) return NULL;
    PyObject* d = NULL;
    /* pickup station */
    if (!(d = PyDict_New())) goto fail;
    for (int i = 0; i < N_PICK; i++)
        if (put(d, s_pick[i], scalar(NPY_INT32, &a[i], 4))) goto fail_d;
    if (put(d, s_mask, vec(NPY_INT8, 3, m, 3))) goto fail_d;
    if (put(obs, s_agents[0], d)) goto fail;
    /* AGV: position = i32[7:9], the other fields i32[9..19] */
    if (!(d = PyDict_New())) goto fail;
    if (put(d, s_agv[0], vec(NPY_INT32, 2, &a[7], 8))) goto fail_d;
    for (int j = 1; j < N_AGV; j++)
        if (put(d, s_agv[j], scalar(NPY_INT32, &a[8 + j], 4))) goto fail_d;
    if (put(d, s_mask, vec(NPY_INT8, 8, &m[3], 8))) goto fail_d;
    if (put(obs, s_agents[1], d)) goto fail;
    /* machines and packaging stations: is_busy i8[2s], processing_progress f32[s], queue_length i8[2s+1] */
    for (int s = 0; s < 6; s++) {
        if (!(d = PyDict_New())) goto fail;
        if (put(d, s_busy, scalar(NPY_INT8, &b[2 * s], 1))) goto fail_d;
        if (put(d, s_prog, scalar(NPY_FLOAT32, &c[s], 4))) goto fail_d;
        if (put(d, s_queue, scalar(NPY_INT8, &b[2 * s + 1], 1))) goto fail_d;
        if (put(d, s_mask, vec(NPY_INT8, 3, &m[MASK_OFF[2 + s]], 3))) goto fail_d;
        if (put(obs, s_agents[2 + s], d)) goto fail;
    }
    return obs;
fail_d:
    Py_DECREF(d);
fail:
    Py_DECREF(obs);
    return NULL;
}

static PyObject* obs_dicts(PyObject* self, PyObject* args) {
    (void)self;
    PyObject *o32, *o8, *of, *om;
    if (!PyArg_ParseTuple(args, "OOOO", &o32, &o8, &of, &om)) return NULL;
    Py_buffer b32, b8, bf, bm;
    if (get_buf(o32, &b32, 20 * 4, "i32")) return NULL;
    if (get_buf(o8, &b8, 12, "i8")) { PyBuffer_Release(&b32); return NULL; }
    if (get_buf(of, &bf, 6 * 4, "f32")) { PyBuffer_Release(&b32); PyBuffer_Release(&b8); return NULL; }
    if (get_buf(om, &bm, 29, "mask")) { PyBuffer_Release(&b32); PyBuffer_Release(&b8); PyBuffer_Release(&bf); return NULL; }
    /* the values are copied out first (the record may be rewritten by the next step only) */
    int32_t a[20];
    int8_t b[12], m[29];
    float c[6];
    memcpy(a, b32.buf, sizeof a);
    memcpy(b, b8.buf, sizeof b);
    memcpy(c, bf.buf, sizeof c);
    memcpy(m, bm.buf, sizeof m);
    PyBuffer_Release(&b32); PyBuffer_Release(&b8); PyBuffer_Release(&bf); PyBuffer_Release(&bm);
    return build_obs(a, b, c, m);
}

/* ---- the fast step */
typedef int (*server_step_fn)(void* h, const uint8_t* actions);
enum { F_I32, F_I8, F_F32, F_MASK, F_REW, F_TERM, F_TRUNC, F_RES, F_OC, F_PK, F_TIME, NF };
typedef struct {
    void* handle;
    server_step_fn fn;
    uint8_t* act;           /* the 8 action bytes handed to the server (pinned host memory) */
    const uint8_t* rec;     /* the step record */
    Py_ssize_t off[NF];     /* field offsets in the record */
    PyObject* cache;        /* dict: i | act << 3 | word << 11 -> decoded action-result dict */
    PyObject* decode;       /* spec.decode_result(agent, action, word) on a cache miss */
} Stepper;

static void stepper_free(PyObject* cap) {
    Stepper* st = (Stepper*)PyCapsule_GetPointer(cap, "fjsp_facade.stepper");
    if (!st) return;
    Py_XDECREF(st->cache);
    Py_XDECREF(st->decode);
    PyMem_Free(st);
}

/* stepper(handle, fn, act_addr, rec_addr, offsets (11 ints: obs_i32, obs_i8, obs_f32, masks,
 * rewards, term, trunc, results, orders_completed, packaged, sim_time), decode) -> capsule */
static PyObject* stepper(PyObject* self, PyObject* args) {
    (void)self;
    unsigned long long h, fn, act, rec;
    PyObject *offs, *decode;
    if (!PyArg_ParseTuple(args, "KKKKOO", &h, &fn, &act, &rec, &offs, &decode)) return NULL;
    if (!h || !fn || !act || !rec) {
        PyErr_SetString(PyExc_ValueError, "stepper: null handle, function or buffer");
        return NULL;
    }
    PyObject* seq = PySequence_Fast(offs, "stepper: offsets must be a sequence");
    if (!seq) return NULL;
    if (PySequence_Fast_GET_SIZE(seq) != NF) {
        Py_DECREF(seq);
        PyErr_SetString(PyExc_ValueError, "stepper: 11 field offsets expected");
        return NULL;
    }
    Stepper* st = (Stepper*)PyMem_Calloc(1, sizeof(Stepper));
    if (!st) { Py_DECREF(seq); return PyErr_NoMemory(); }
    for (int i = 0; i < NF; i++) {
        st->off[i] = PyLong_AsSsize_t(PySequence_Fast_GET_ITEM(seq, i));
        if (st->off[i] < 0) {
            Py_DECREF(seq);
            PyMem_Free(st);
            if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "stepper: negative offset");
            return NULL;
        }
    }
    Py_DECREF(seq);
    st->handle = (void*)(uintptr_t)h;
    st->fn = (server_step_fn)(uintptr_t)fn;
    st->act = (uint8_t*)(uintptr_t)act;
    st->rec = (const uint8_t*)(uintptr_t)rec;
    if (!(st->cache = PyDict_New())) { PyMem_Free(st); return NULL; }
    Py_INCREF(decode);
    st->decode = decode;
    PyObject* cap = PyCapsule_New(st, "fjsp_facade.stepper", stepper_free);
    if (!cap) { Py_DECREF(st->cache); Py_DECREF(decode); PyMem_Free(st); }
    return cap;
}

static PyObject* bool_dict(int v) {
    PyObject* d = PyDict_New();
    if (!d) return NULL;
    for (int i = 0; i < N_AG; i++)
        if (PyDict_SetItem(d, s_agents[i], v ? Py_True : Py_False)) { Py_DECREF(d); return NULL; }
    return d;
}

/* step(stepper, actions) -> None (not the common case: nothing done), an int (the server's
 * nonzero return code), or (obs, rewards, terms, truncs, infos, sim_time, packaged) */
static PyObject* step(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
    (void)self;
    if (nargs != 2) {
        PyErr_SetString(PyExc_TypeError, "step(stepper, actions)");
        return NULL;
    }
    Stepper* st = (Stepper*)PyCapsule_GetPointer(args[0], "fjsp_facade.stepper");
    if (!st) return NULL;
    PyObject* actions = args[1];
    if (!PyDict_CheckExact(actions) || PyDict_GET_SIZE(actions) != N_AG) Py_RETURN_NONE;
    /* the canonical dict order with plain ints 0..253 (FJSPSimulation.step's fast codes) */
    uint8_t codes[N_AG];
    long acts[N_AG];
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    for (int i = 0; PyDict_Next(actions, &pos, &k, &v); i++) {
        if (k != s_agents[i] && (!PyUnicode_CheckExact(k) || PyUnicode_Compare(k, s_agents[i]) != 0)) {
            if (PyErr_Occurred()) PyErr_Clear();
            Py_RETURN_NONE;
        }
        if (!PyLong_CheckExact(v)) Py_RETURN_NONE;
        int overflow = 0;
        const long x = PyLong_AsLongAndOverflow(v, &overflow);
        if (overflow || x < 0 || x > 253) {
            if (PyErr_Occurred()) PyErr_Clear();
            Py_RETURN_NONE;
        }
        codes[i] = (uint8_t)x;
        acts[i] = x;
    }
    memcpy(st->act, codes, N_AG);
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = st->fn(st->handle, st->act);   /* returns with the step's record written */
    Py_END_ALLOW_THREADS
    if (rc != 0) return PyLong_FromLong(rc);
    const uint8_t* r = st->rec;
    int32_t a[20];
    int8_t b[12], m[29];
    float c[6];
    double rew[N_AG], sim_time;
    uint32_t res[N_AG];
    int32_t oc, pk;
    memcpy(a, r + st->off[F_I32], sizeof a);
    memcpy(b, r + st->off[F_I8], sizeof b);
    memcpy(c, r + st->off[F_F32], sizeof c);
    memcpy(m, r + st->off[F_MASK], sizeof m);
    memcpy(rew, r + st->off[F_REW], sizeof rew);
    memcpy(res, r + st->off[F_RES], sizeof res);
    memcpy(&oc, r + st->off[F_OC], 4);
    memcpy(&pk, r + st->off[F_PK], 4);
    memcpy(&sim_time, r + st->off[F_TIME], 8);
    const int term = r[st->off[F_TERM]] != 0, trunc = r[st->off[F_TRUNC]] != 0;

    PyObject *obs = NULL, *rewards = NULL, *terms = NULL, *truncs = NULL, *infos = NULL;
    PyObject *t_time = NULL, *t_oc = NULL, *t_pk = NULL, *out = NULL;
    if (!(obs = build_obs(a, b, c, m))) goto done;
    if (!(rewards = PyDict_New())) goto done;
    for (int i = 0; i < N_AG; i++)
        if (put(rewards, s_agents[i], PyFloat_FromDouble(rew[i]))) goto done;
    if (!(terms = bool_dict(term)) || !(truncs = bool_dict(trunc))) goto done;
    if (!(t_time = PyFloat_FromDouble(sim_time)) || !(t_oc = PyLong_FromLong(oc)) || !(t_pk = PyLong_FromLong(pk)))
        goto done;
    if (!(infos = PyDict_New())) goto done;
    for (int i = 0; i < N_AG; i++) {
        PyObject* key = PyLong_FromUnsignedLongLong((unsigned long long)i | ((unsigned long long)acts[i] << 3) |
                                                    ((unsigned long long)res[i] << 11));
        if (!key) goto done;
        PyObject* dec = PyDict_GetItemWithError(st->cache, key);   /* borrowed */
        if (!dec) {
            if (PyErr_Occurred()) { Py_DECREF(key); goto done; }
            dec = PyObject_CallFunction(st->decode, "OlI", s_agents[i], acts[i], (unsigned int)res[i]);
            if (!dec || PyDict_SetItem(st->cache, key, dec)) { Py_XDECREF(dec); Py_DECREF(key); goto done; }
            Py_DECREF(dec);   /* the cache holds it */
            dec = PyDict_GetItem(st->cache, key);
        }
        Py_DECREF(key);
        PyObject* ar = PyDict_Copy(dec);
        PyObject* d = ar ? PyDict_New() : NULL;
        if (!d || put(d, s_ares, ar) || PyDict_SetItem(d, s_stime, t_time) || PyDict_SetItem(d, s_ocomp, t_oc) ||
            PyDict_SetItem(d, s_tpack, t_pk) || put(infos, s_agents[i], d)) {
            if (!d) Py_XDECREF(ar);
            goto done;
        }
    }
    out = PyTuple_Pack(7, obs, rewards, terms, truncs, infos, t_time, t_pk);
done:
    Py_XDECREF(obs); Py_XDECREF(rewards); Py_XDECREF(terms); Py_XDECREF(truncs); Py_XDECREF(infos);
    Py_XDECREF(t_time); Py_XDECREF(t_oc); Py_XDECREF(t_pk);
    return out;
}

static PyMethodDef methods[] = {
    {"obs_dicts", obs_dicts, METH_VARARGS,
     "obs_dicts(i32, i8, f32, mask) -> the reference's observation dict of one env (spec.obs_dicts)"},
    {"stepper", stepper, METH_VARARGS,
     "stepper(handle, server_step_actions, act_addr, record_addr, offsets, decode) -> a step configuration"},
    {"step", (PyCFunction)(void (*)(void))step, METH_FASTCALL,
     "step(stepper, actions) -> None | rc | (obs, rewards, terms, truncs, infos, sim_time, packaged)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_facade", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__facade(void) {
    import_array();
    for (int i = 0; i < N_AG; i++)
        if (!(s_agents[i] = PyUnicode_InternFromString(AGENTS[i]))) return NULL;
    for (int i = 0; i < N_PICK; i++)
        if (!(s_pick[i] = PyUnicode_InternFromString(PICK[i]))) return NULL;
    for (int i = 0; i < N_AGV; i++)
        if (!(s_agv[i] = PyUnicode_InternFromString(AGV[i]))) return NULL;
    if (!(s_busy = PyUnicode_InternFromString("is_busy")) || !(s_prog = PyUnicode_InternFromString("processing_progress")) ||
        !(s_queue = PyUnicode_InternFromString("queue_length")) || !(s_mask = PyUnicode_InternFromString("action_mask")) ||
        !(s_ares = PyUnicode_InternFromString("action_result")) || !(s_stime = PyUnicode_InternFromString("sim_time")) ||
        !(s_ocomp = PyUnicode_InternFromString("orders_completed")) ||
        !(s_tpack = PyUnicode_InternFromString("total_products_packaged")))
        return NULL;
    return PyModule_Create(&module);
}
