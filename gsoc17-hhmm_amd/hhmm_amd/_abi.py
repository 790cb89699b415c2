"""ctypes mirror of include/hhmm.h (ABI version 2).

Field order and types must match the C structs exactly; tests/test_abi.py
checks the sizes against offsets parsed from the header.
"""
import ctypes as C

ABI_VERSION = 2

# hhmm_status
OK = 0
WARN_PAIR_FAILURES = 1
ERR_INVALID_ARGUMENT = -1
ERR_OUT_OF_MEMORY = -2
ERR_HIP = -3
ERR_UNSUPPORTED = -4
ERR_NO_DEVICE = -5

PAIR_OK = 0
PAIR_INVALID_BACKPOINTER = 1
PAIR_INVALID_DATA = 2  # hhmm_run_device: the series breaks a data-block bound (include/hhmm.h)

MODELS = {
    "hmm": 1,                    # hmm/stan/hmm.stan
    "hmm-multinom": 2,           # hmm/stan/hmm-multinom.stan
    "hmm-multinom-semisup": 3,   # hmm/stan/hmm-multinom-semisup.stan
    "iohmm-reg": 4,              # iohmm-reg/stan/iohmm-reg.stan
    "iohmm-mix": 5,              # iohmm-mix/stan/iohmm-mix.stan
    "iohmm-hmix": 6,             # iohmm-mix/stan/iohmm-hmix.stan
    "iohmm-hmix-lite": 7,        # iohmm-mix/stan/iohmm-hmix-lite.stan
    "hhmm-tayal2009": 8,         # tayal2009/stan/hhmm-tayal2009.stan
    "hhmm-tayal2009-lite": 9,    # tayal2009/stan/hhmm-tayal2009-lite.stan
}

PAIR_GRID = 0
PAIR_ZIP = 1
PAIR_BLOCK = 2

# hhmm_request.flags
FLAG_SCAN_AUTO = 0
FLAG_SCAN_FORCE = 1 << 0
FLAG_SCAN_OFF = 1 << 1
FLAG_NO_FUSE = 1 << 2
FLAG_VIT_LANES = 1 << 3
FLAG_VIT_STATES = 1 << 4
FLAG_FUSED = 1 << 5
FLAG_VIT_SCAN = 1 << 6
FLAG_VIT_SCAN_OFF = 1 << 7
FLAG_FB_SPLIT = 1 << 16
FLAG_LKM_MFMA = 1 << 17
FLAG_VFB = 1 << 18
FLAG_VFB_OFF = 1 << 19
DEVICE_SET = -2  # hhmm_request.device: shard over the device set (HHMM_DEVICE_SET)


def flag_scan_chunk_log2(n):
    """T-chunk length 2^n for the parallel scan (HHMM_FLAG_SCAN_CHUNK_LOG2)."""
    return int(n) << 8


def flag_host_chunks(n):
    """hhmm_run's host pipeline in n chunks (HHMM_FLAG_HOST_CHUNKS; 0 = automatic)."""
    return (int(n) & 0xFF) << 20

OUT = {
    "loglik": 1 << 0,
    "unalpha_tk": 1 << 1,
    "alpha_tk": 1 << 2,
    "unbeta_tk": 1 << 3,
    "beta_tk": 1 << 4,
    "ungamma_tk": 1 << 5,
    "gamma_tk": 1 << 6,
    "zstar_t": 1 << 7,
    "logp_zstar": 1 << 8,
    "oblik_tk": 1 << 9,
    "oblik_t": 1 << 10,
    "z_ffbs": 1 << 11,
    "alpha_tk_oos": 1 << 12,
    "unalpha_tk_oos": 1 << 13,
    "logA_ij": 1 << 14,
    "hatpi_tk": 1 << 15,
    "hatz_t": 1 << 16,
    "hatl_t": 1 << 17,
    "hatx_t": 1 << 18,
}

I32P = C.POINTER(C.c_int32)
F64P = C.POINTER(C.c_double)


class Data(C.Structure):
    _fields_ = [
        ("n_series", C.c_int64),
        ("T_max", C.c_int32),
        ("K", C.c_int32),
        ("L", C.c_int32),
        ("M", C.c_int32),
        ("G", C.c_int32),
        ("T_oos_max", C.c_int32),
        ("T", C.c_void_p),
        ("x_int", C.c_void_p),
        ("x_real", C.c_void_p),
        ("g", C.c_void_p),
        ("sign", C.c_void_p),
        ("u", C.c_void_p),
        ("T_oos", C.c_void_p),
        ("x_oos", C.c_void_p),
        ("sign_oos", C.c_void_p),
        ("hyperparams", C.c_void_p),
    ]


class Draws(C.Structure):
    _fields_ = [
        ("n_draws", C.c_int64),
        ("p_1k", C.c_void_p),
        ("A_ij", C.c_void_p),
        ("phi_k", C.c_void_p),
        ("mu_k", C.c_void_p),
        ("sigma_k", C.c_void_p),
        ("w_km", C.c_void_p),
        ("b_km", C.c_void_p),
        ("s_k", C.c_void_p),
        ("lambda_kl", C.c_void_p),
        ("mu_kl", C.c_void_p),
        ("s_kl", C.c_void_p),
        ("p_11", C.c_void_p),
        ("A_row", C.c_void_p),
    ]


class Request(C.Structure):
    _fields_ = [
        ("abi_version", C.c_uint32),
        ("model", C.c_int32),
        ("pairing", C.c_int32),
        ("outputs", C.c_uint32),
        ("data", Data),
        ("draws", Draws),
        ("ffbs_u", C.c_void_p),
        ("device", C.c_int32),
        ("flags", C.c_int32),
        ("hat_rand", C.c_void_p),
    ]


class Result(C.Structure):
    _fields_ = [
        ("loglik", C.c_void_p),
        ("unalpha_tk", C.c_void_p),
        ("alpha_tk", C.c_void_p),
        ("unbeta_tk", C.c_void_p),
        ("beta_tk", C.c_void_p),
        ("ungamma_tk", C.c_void_p),
        ("gamma_tk", C.c_void_p),
        ("zstar_t", C.c_void_p),
        ("logp_zstar", C.c_void_p),
        ("oblik_tk", C.c_void_p),
        ("oblik_t", C.c_void_p),
        ("z_ffbs", C.c_void_p),
        ("alpha_tk_oos", C.c_void_p),
        ("unalpha_tk_oos", C.c_void_p),
        ("logA_ij", C.c_void_p),
        ("pair_status", C.c_void_p),
        ("hatpi_tk", C.c_void_p),
        ("hatz_t", C.c_void_p),
        ("hatl_t", C.c_void_p),
        ("hatx_t", C.c_void_p),
    ]


# Data-block fields (name -> (ctype kind, shape code)).  Shape codes use
# N = series, T = T_max, M, To = T_oos_max.
DATA_ARRAYS = {
    "T": ("i32", "N"),
    "x_int": ("i32", "NT"),
    "x_real": ("f64", "NT"),
    "g": ("i32", "NT"),
    "sign": ("i32", "NT"),
    "u": ("f64", "NTM"),
    "T_oos": ("i32", "N"),
    "x_oos": ("i32", "NTo"),
    "sign_oos": ("i32", "NTo"),
    "hyperparams": ("f64", "9"),
}

DRAW_ARRAYS = {
    "p_1k": "SK",
    "A_ij": "SKK",
    "phi_k": "SKL",
    "mu_k": "SK",
    "sigma_k": "SK",
    "w_km": "SKM",
    "b_km": "SKM",
    "s_k": "SK",
    "lambda_kl": "SKL",
    "mu_kl": "SKL",
    "s_kl": "SKL",
    "p_11": "S",
    "A_row": "S22",
}

# result field -> (dtype, shape code) ; P = pairs
RESULT_ARRAYS = {
    "loglik": ("f64", "P"),
    "unalpha_tk": ("f64", "PTK"),
    "alpha_tk": ("f64", "PTK"),
    "unbeta_tk": ("f64", "PTK"),
    "beta_tk": ("f64", "PTK"),
    "ungamma_tk": ("f64", "PTK"),
    "gamma_tk": ("f64", "PTK"),
    "zstar_t": ("i32", "PTz"),
    "logp_zstar": ("f64", "P"),
    "oblik_tk": ("f64", "PTK"),
    "oblik_t": ("f64", "PT"),
    "z_ffbs": ("i32", "PT"),
    "alpha_tk_oos": ("f64", "PToK"),
    "unalpha_tk_oos": ("f64", "PToK"),
    "logA_ij": ("f64", "PTK"),
    "hatpi_tk": ("f64", "PTK"),
    "hatz_t": ("i32", "PT"),
    "hatl_t": ("i32", "PT"),
    "hatx_t": ("f64", "PT"),
}


def declare(lib):
    """Attach argtypes / restypes of the public entry points."""
    RP = C.POINTER(Request)
    SP = C.POINTER(Result)
    lib.hhmm_version.restype = C.c_char_p
    lib.hhmm_last_error.restype = C.c_char_p
    lib.hhmm_num_pairs.argtypes = [RP]
    lib.hhmm_num_pairs.restype = C.c_int64
    lib.hhmm_validate.argtypes = [RP, SP, C.c_int]
    lib.hhmm_validate.restype = C.c_int
    lib.hhmm_init.argtypes = [C.c_int]
    lib.hhmm_init.restype = C.c_int
    lib.hhmm_shutdown.restype = C.c_int
    if hasattr(lib, "hhmm_init_devices"):  # absent from libraries built before the device set (A/B variants)
        lib.hhmm_init_devices.argtypes = [C.POINTER(C.c_int32), C.c_int]
        lib.hhmm_init_devices.restype = C.c_int
        lib.hhmm_device_set.argtypes = [C.POINTER(C.c_int32), C.c_int]
        lib.hhmm_device_set.restype = C.c_int
    lib.hhmm_run.argtypes = [RP, SP]
    lib.hhmm_run.restype = C.c_int
    lib.hhmm_workspace_size.argtypes = [RP, C.POINTER(C.c_size_t)]
    lib.hhmm_workspace_size.restype = C.c_int
    lib.hhmm_run_device.argtypes = [RP, SP, C.c_void_p, C.c_size_t, C.c_void_p]
    lib.hhmm_run_device.restype = C.c_int
    lib.hhmm_selftest_cr_log.argtypes = [F64P, F64P, C.c_int64]
    lib.hhmm_selftest_cr_log.restype = C.c_int
    lib.hhmm_selftest_cr_exp.argtypes = [F64P, F64P, C.c_int64]
    lib.hhmm_selftest_cr_exp.restype = C.c_int
    lib.hhmm_selftest_det_log.argtypes = [F64P, F64P, C.c_int64]
    lib.hhmm_selftest_det_log.restype = C.c_int
    lib.hhmm_selftest_det_exp.argtypes = [F64P, F64P, C.c_int64]
    lib.hhmm_selftest_det_exp.restype = C.c_int
    lib.hhmm_selftest_shards.argtypes = [RP, SP, C.c_int]
    lib.hhmm_selftest_shards.restype = C.c_int
    lib.hhmm_selftest_pipeline.argtypes = [RP, SP, C.c_int, C.c_int]
    lib.hhmm_selftest_pipeline.restype = C.c_int
    return lib
