"""ctypes binding of libfjsp.so (C-ABI declared in include/fjsp.h).

The library is the ONLY compute path of this package: every reset / step / GAE call goes to
the HIP kernels for gfx950.  If the library is missing or no GPU is visible, the calls fail
loudly (FjspNativeError) — there is no CPU fallback.
"""
import ctypes
import importlib
import os
import subprocess
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
# FJSP_LIB selects a diagnostic build (e.g. libfjsp_stamps.so); default: the product library
LIB_PATH = os.environ.get("FJSP_LIB") or os.path.join(HERE, "libfjsp.so")
SRC = os.path.join(HERE, "csrc", "fjsp_hip.hip")
SRCS = [SRC, os.path.join(HERE, "csrc", "fjsp_policy.hip"), os.path.join(HERE, "csrc", "fjsp_group.hip")]
HEADERS = [os.path.join(HERE, "csrc", h) for h in ("fjsp_env.h", "fjsp_stepdev.h", "fjsp_stamps.h")] + [
    os.path.join(REPO, "include", "fjsp.h")]

# the drop-in facade's host helper (CPython extension, no GPU code): csrc/fjsp_facade.c
FACADE_SRC = os.path.join(HERE, "csrc", "fjsp_facade.c")
FACADE_PATH = os.path.join(HERE, "_facade" + sysconfig.get_config_var("EXT_SUFFIX"))

HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-ffp-contract=off", "-Wall", "-Wno-unused-function"]


class FjspNativeError(RuntimeError):
    pass


class fjsp_config(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int32) for k in (
        "num_trays", "tray_capacity", "mask_tray_capacity", "storage_capacity", "step_size",
        "max_episode_steps", "agv_speed", "pt_small", "pt_big", "pt_packaging", "packaging_capacity")]


REWARD_FIELDS = ["order_complete_reward", "throughput_bonus", "time_penalty", "pickup_load_reward",
                 "pickup_tray_complete", "pickup_idle_penalty", "agv_delivery_reward", "agv_move_penalty",
                 "agv_packaging_delivery", "agv_invalid_action", "machine_complete_reward", "machine_start_reward",
                 "machine_idle_penalty", "packaging_complete_reward", "packaging_start_reward",
                 "packaging_idle_penalty"]


class fjsp_reward_weights(ctypes.Structure):
    _fields_ = [(k, ctypes.c_double) for k in REWARD_FIELDS]


OUT_FIELDS = ["obs_i32", "obs_i8", "obs_f32", "masks", "rewards", "term", "trunc", "results",
              "orders_completed", "packaged", "sim_time", "status",
              "next_i32", "next_i8", "next_f32", "next_masks", "feats"]


class fjsp_out(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k in OUT_FIELDS]


class fjsp_env_view(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int32) for k in (
        "current_step", "num_orders", "next_order", "orders_completed", "total_packaged",
        "agv_row", "agv_col", "agv_carrying", "agv_tray_count")] + [
        ("status", ctypes.c_uint32), ("orders", ctypes.c_uint32 * 64)]


# every symbol include/fjsp.h declares (checked by tests/test_abi.py)
EXPORTS = ["fjsp_abi_version", "fjsp_last_error", "fjsp_default_config", "fjsp_check_config",
           "fjsp_default_reward_weights", "fjsp_set_reward_weights",
           "fjsp_create", "fjsp_destroy", "fjsp_set_stream", "fjsp_set_option", "fjsp_num_envs", "fjsp_state_bytes",
           "fjsp_reset", "fjsp_step", "fjsp_step_many", "fjsp_gae", "fjsp_gae_f64", "fjsp_mt_get", "fjsp_mt_set",
           "fjsp_read_env", "fjsp_sync", "fjsp_last_kernel_ms", "fjsp_pack_a2c", "fjsp_a2c_layout",
           "fjsp_snapshot_bytes", "fjsp_snapshot", "fjsp_restore", "fjsp_last_kernel", "fjsp_a2c_policy",
           "fjsp_a2c_group_keys", "fjsp_a2c_group_verify", "fjsp_a2c_actor_head",
           "fjsp_a2c_relu_bias_grad", "fjsp_a2c_value_head_grad", "fjsp_faults", "fjsp_a2c_critic_forward",
           "fjsp_a2c_critic_backward", "fjsp_gae_shared",
           "fjsp_a2c_policy_step", "fjsp_a2c_group_temp_bytes", "fjsp_a2c_group_sort", "fjsp_a2c_group_runs",
           "fjsp_a2c_run_sums_bytes", "fjsp_a2c_run_sums", "fjsp_a2c_critic_fused", "fjsp_a2c_shard_keys", "fjsp_a2c_record_head", "fjsp_a2c_pack_mfma", "fjsp_a2c_slab_stats",
           "fjsp_a2c_wgrad", "fjsp_server_start", "fjsp_server_step", "fjsp_server_step_actions", "fjsp_server_stop"]
POLICY_ACTOR_DPAD, POLICY_CRITIC_DPAD = 16, 48
POLICY_ACTOR_FLOATS = 3 * 256 * 16 // 2 + 256 + 3 * 256 * 256 // 2 + 256 + 8 * 256 + 16
POLICY_CRITIC_FLOATS = 3 * 256 * 48 // 2 + 256 + 3 * 256 * 256 // 2 + 256 + 3 * 128 * 256 // 2 + 128 + 128 + 16
CRITIC_FUSED_PW = 2 * 256 + 2 * 128 + 4   # floats per tile of fjsp_a2c_critic_fused's partial sums
ABI_VERSION = 12

_lib = None


def _stale():
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.getmtime(p) > t for p in SRCS + HEADERS)


def build_facade(force=False):
    """Compile the facade's CPython helper (_facade*.so) in-tree with gcc."""
    if not force and os.path.exists(FACADE_PATH) and os.path.getmtime(FACADE_PATH) >= os.path.getmtime(FACADE_SRC):
        return FACADE_PATH
    import numpy
    r = subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-Wall", "-Wextra", "-Wno-unused-parameter",
                        "-I" + sysconfig.get_paths()["include"], "-I" + numpy.get_include(), "-o", FACADE_PATH,
                        FACADE_SRC], capture_output=True, text=True)
    if r.returncode != 0:
        raise FjspNativeError("gcc failed on fjsp_facade.c:\n" + r.stderr[-4000:])
    return FACADE_PATH


def facade():
    """The facade's host helper module (obs_dicts in C); fails loudly when it was not built."""
    if not os.path.exists(FACADE_PATH):
        raise FjspNativeError(
            f"{FACADE_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    return importlib.import_module(__package__ + "._facade")


def build(force=False, verbose=False):
    """Compile libfjsp.so for gfx950 in-tree (hipcc cross-compiles without a GPU): one hipcc
    process per source file in parallel (no cross-file device calls), then one link; and the
    facade's host helper."""
    build_facade(force)
    if not force and not _stale():
        return LIB_PATH
    import tempfile
    with tempfile.TemporaryDirectory(prefix="fjsp_build_") as tmp:
        objs = [os.path.join(tmp, os.path.basename(s) + ".o") for s in SRCS]
        cflags = [f for f in HIPCC_FLAGS if f != "-shared"]
        procs = [subprocess.Popen(["hipcc"] + cflags + ["-c", "-o", o, s], stdout=subprocess.PIPE,
                                  stderr=subprocess.PIPE, text=True) for s, o in zip(SRCS, objs)]
        errs = []
        for p in procs:
            _, err = p.communicate()
            if p.returncode != 0:
                errs.append(err)
            elif verbose and err:
                print(err)
        if errs:
            raise FjspNativeError("hipcc failed:\n" + "\n".join(e[-4000:] for e in errs))
        r = subprocess.run(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB_PATH] + objs,
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise FjspNativeError("hipcc link failed:\n" + r.stderr[-4000:])
    return LIB_PATH


def lib():
    """Load libfjsp.so (after torch, so one HIP runtime serves both)."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  (loads torch's libamdhip64 first: same SONAME -> shared runtime)
    if not os.path.exists(LIB_PATH):
        raise FjspNativeError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(LIB_PATH)
    P, I, U32, U64, D = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_double
    sig = {
        "fjsp_abi_version": (I, []),
        "fjsp_last_error": (ctypes.c_char_p, []),
        "fjsp_default_config": (I, [ctypes.POINTER(fjsp_config)]),
        "fjsp_check_config": (I, [ctypes.POINTER(fjsp_config)]),
        "fjsp_default_reward_weights": (I, [ctypes.POINTER(fjsp_reward_weights)]),
        "fjsp_set_reward_weights": (I, [P, ctypes.POINTER(fjsp_reward_weights)]),
        "fjsp_create": (I, [ctypes.POINTER(fjsp_config), I, I, P, ctypes.POINTER(P)]),
        "fjsp_destroy": (I, [P]),
        "fjsp_set_stream": (I, [P, P]),
        "fjsp_set_option": (I, [P, ctypes.c_char_p, ctypes.c_int64]),
        "fjsp_num_envs": (I, [P]),
        "fjsp_state_bytes": (ctypes.c_int64, [P]),
        "fjsp_reset": (I, [P, P, P, I, ctypes.POINTER(fjsp_out)]),
        "fjsp_step": (I, [P, P, P, I, ctypes.POINTER(fjsp_out)]),
        "fjsp_step_many": (I, [P, I, U64, U32, U32, I, I, ctypes.POINTER(fjsp_out)]),
        "fjsp_gae": (I, [P, P, P, P, I, I, I, D, D, P, P, P]),
        "fjsp_gae_f64": (I, [P, P, P, P, I, I, I, D, D, P, P, P]),
        "fjsp_mt_get": (I, [P, I, P, ctypes.POINTER(I)]),
        "fjsp_mt_set": (I, [P, I, P, I]),
        "fjsp_read_env": (I, [P, I, ctypes.POINTER(fjsp_env_view)]),
        "fjsp_sync": (I, [P]),
        "fjsp_last_kernel_ms": (I, [P, ctypes.POINTER(ctypes.c_float)]),
        "fjsp_pack_a2c": (I, [P, P, P]),
        "fjsp_a2c_layout": (I, [P]),
        "fjsp_snapshot_bytes": (ctypes.c_int64, [P]),
        "fjsp_snapshot": (I, [P, P]),
        "fjsp_restore": (I, [P, P]),
        "fjsp_last_kernel": (ctypes.c_char_p, [P]),
        "fjsp_faults": (I, [P, ctypes.POINTER(U32), I]),
        "fjsp_a2c_policy": (I, [P, P, I, P, P, P, U32, U32, I, P, P, P, P]),
        "fjsp_a2c_group_keys": (I, [P, I, I, P, P, P]),
        "fjsp_a2c_group_verify": (I, [P, I, I, P, P, P, P]),
        "fjsp_a2c_relu_bias_grad": (I, [P, P, ctypes.c_int64, I, P, P, P]),
        "fjsp_a2c_value_head_grad": (I, [P, P, P, ctypes.c_int64, P, P, P]),
        "fjsp_a2c_actor_head": (I, [P, I, P, I, I, P, P, P, P, P, ctypes.c_float, ctypes.c_float, P, P, P]),
        "fjsp_a2c_critic_forward": (I, [P, I, P, P, P, P, P, P]),
        "fjsp_a2c_critic_backward": (I, [P, P, P, I, P, P, P, P, P, P, P]),
        "fjsp_gae_shared": (I, [P, P, P, I, I, I, D, D, P, P, P]),
        "fjsp_a2c_policy_step": (I, [P, P, P, P, P, P, U32, U32, I, P, P, I, ctypes.POINTER(fjsp_out), I, I, P]),
        "fjsp_server_start": (I, [P, P, I, ctypes.POINTER(fjsp_out)]),
        "fjsp_server_step": (I, [P]),
        "fjsp_server_step_actions": (I, [P, P]),
        "fjsp_server_stop": (I, [P]),
        "fjsp_a2c_group_temp_bytes": (I, [ctypes.c_int64, ctypes.POINTER(U64)]),
        "fjsp_a2c_group_sort": (I, [P, I, ctypes.c_int64, ctypes.c_uint32, P, U64, P, P, P, P, P, P, P, P]),
        "fjsp_a2c_group_runs": (I, [P, P, I, ctypes.c_int64, ctypes.c_int64, P, P, P, P, P, P, P, P]),
        "fjsp_a2c_run_sums_bytes": (I, [I, ctypes.c_int64, ctypes.POINTER(U64)]),
        "fjsp_a2c_run_sums": (I, [P, I, P, P, P, P, ctypes.c_int64, ctypes.c_int64, P, U64, P, P]),
        "fjsp_a2c_critic_fused": (I, [P, I, P, P, P, P, P, P, P, P, P, P, P, P, P]),
        "fjsp_a2c_shard_keys": (I, [P, P, P, I, I, P, P, P, P]),
        "fjsp_a2c_record_head": (I, [P, I, P, I, I, P, P, P, ctypes.c_float, ctypes.c_float, P, P, P]),
        "fjsp_a2c_pack_mfma": (I, [P, I, I, I, I, P, P]),
        "fjsp_a2c_slab_stats": (I, [P, P, I, I, P, P, P, P]),
        "fjsp_a2c_wgrad": (I, [P, I, ctypes.c_int64, P, I, ctypes.c_int64, ctypes.c_int64, P, I, P, I, ctypes.c_int64, P]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.fjsp_abi_version() != ABI_VERSION:
        raise FjspNativeError("libfjsp.so ABI version mismatch")
    _lib = L
    return L


def check(rc):
    if rc != 0:
        raise FjspNativeError(lib().fjsp_last_error().decode())
    return rc


def default_config(**over):
    c = fjsp_config()
    lib().fjsp_default_config(ctypes.byref(c))
    for k, v in over.items():
        setattr(c, k, int(v))
    return c
