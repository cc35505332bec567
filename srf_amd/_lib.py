"""ctypes binding of the C ABI in ``include/srf.h`` (``srf_amd/libsrf.so``).

The library is the only compute path for the routing layers: there is no CPU
or eager-PyTorch fallback, so a missing or stale build raises here instead of
silently running something else.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('SRF_LIB_PATH') or os.path.join(_HERE, 'libsrf.so')   # override: A/B builds

_c_int, _c_size, _vp = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p

SDR_MAX_ITEMS = 8   # SRF_SDR_MAX_ITEMS


class SdrRange(ctypes.Structure):
    """srf_sdr_range: one frame range of one SDR layer for the batched entry points."""
    _fields_ = [('t0', _c_int), ('t1', _c_int), ('emb', _vp), ('W', _vp), ('bias', _vp), ('WT', _vp),
                ('u', _vp), ('v0', _c_int), ('vn', _c_int), ('v', _vp), ('couplings', _vp),
                ('workspace', _vp), ('workspace_bytes', _c_size), ('g_v', _vp), ('carry', _vp),
                ('gu', _vp), ('g0', _c_int), ('gn', _c_int), ('g_emb', _vp), ('g_W', _vp), ('g_bias', _vp),
                ('accumulate', _c_int), ('u_bf16', _c_int), ('group', _c_int), ('gu_factored', _c_int)]


_ranges = ctypes.POINTER(SdrRange)

CAPSNORM_MAX_ITEMS = 8   # SRF_CAPSNORM_MAX_ITEMS


class CapsnormRange(ctypes.Structure):
    """srf_capsnorm_range: one layer's frame range for srf_capsnorm_{fwd,bwd}_range_n."""
    _fields_ = [('t0', _c_int), ('t1', _c_int), ('layer', _c_int), ('x', _vp), ('gamma', _vp), ('beta', _vp),
                ('y', _vp), ('stat', _vp), ('g_y', _vp), ('g_x', _vp), ('gpart', _vp)]


_cn_ranges = ctypes.POINTER(CapsnormRange)

# name -> (restype, argtypes); mirrors include/srf.h one to one.
_SIGNATURES = {
    'srf_version': (_c_int, []),
    'srf_last_error': (ctypes.c_char_p, []),
    'srf_set_seed_source': (_c_int, [_vp]),
    'srf_set_fault_flag': (_c_int, [_vp]),
    'srf_route_dr_auto_chunks': (_c_int, [_c_int] * 8),
    'srf_route_dr_saved_floats': (_c_size, [_c_int] * 5),
    'srf_route_dr_fwd_workspace': (_c_size, [_c_int] * 10),
    'srf_route_dr_bwd_workspace': (_c_size, [_c_int] * 10),
    'srf_route_dr_fwd': (_c_int, [_vp, _vp, _vp] + [_c_int] * 11 + [_vp, _vp, _vp, _c_size, _vp]),
    'srf_route_dr_bwd': (_c_int, [_vp, _vp, _vp] + [_c_int] * 11 + [_vp, _vp, _vp, _vp, _vp, _vp, _c_size, _vp]),
    'srf_route_dr_bwd_data': (_c_int, [_vp, _vp, _vp] + [_c_int] * 11 + [_vp, _vp, _vp, _vp, _c_size, _vp]),
    'srf_route_dr_bwd_weights': (_c_int, [_vp] + [_c_int] * 11 + [_vp, _vp, _vp, _c_size, _vp]),
    'srf_route_dr_coupling_floats': (_c_size, [_c_int] * 9),
    'srf_route_dr_fwd_ex': (_c_int, [_vp, _vp, _vp] + [_c_int] * 11 + [_vp, _vp, _vp, _vp, _c_size, _vp]),
    'srf_route_dr_bwd_ex': (_c_int, [_vp, _vp, _vp] + [_c_int] * 11 + [_vp] * 7 + [_c_size, _vp]),
    'srf_route_dr_bwd_data_ex': (_c_int, [_vp, _vp, _vp] + [_c_int] * 11 + [_vp] * 5 + [_c_size, _vp]),
    'srf_route_dr_bwd_weights_ex': (_c_int, [_vp] + [_c_int] * 11 + [_vp] * 5 + [_c_size, _vp]),
    'srf_route_sdr_saved_floats': (_c_size, [_c_int] * 4),
    'srf_route_sdr_fwd_workspace': (_c_size, [_c_int] * 8),
    'srf_route_sdr_bwd_workspace': (_c_size, [_c_int] * 9),
    'srf_route_sdr_fwd': (_c_int, [_vp, _vp, _vp] + [_c_int] * 10 + [_vp, _vp, _vp, _c_size, _vp]),
    'srf_route_sdr_bwd': (_c_int, [_vp, _vp, _vp] + [_c_int] * 10 + [_vp, _vp, _vp, _vp, _vp, _vp, _c_size, _vp]),
    'srf_route_sdr_pose': (_c_int, [_vp, _vp, _vp] + [_c_int] * 10 + [_vp, _c_int, _c_int, _vp]),
    'srf_route_sdr_pose_fp8': (_c_int, [_vp, _vp, _vp] + [_c_int] * 10 + [_vp, _c_int, _c_int, _vp]),
    'srf_route_sdr_recur_workspace': (_c_size, [_c_int] * 5),
    'srf_route_sdr_recur_zero_range': (_c_size, [_c_int] * 5 + [ctypes.POINTER(_c_size)]),
    'srf_route_sdr_coupling_floats': (_c_size, [_c_int] * 4),
    'srf_route_sdr_couplings_required': (_c_int, [_c_int] * 4),
    'srf_route_sdr_fact_floats': (_c_size, [_c_int] * 4),
    'srf_route_sdr_recur_fwd': (_c_int, [_vp] + [_c_int] * 11 + [_vp, _vp, _vp, _c_size, _vp]),
    'srf_route_sdr_recur_bwd': (_c_int, [_vp, _c_int, _c_int, _vp, _vp, _vp] + [_c_int] * 9
                                + [_vp, _vp, _c_int, _c_int, _vp, _c_size, _vp]),
    'srf_route_sdr_transpose_w': (_c_int, [_vp] + [_c_int] * 4 + [_vp, _vp]),
    'srf_route_sdr_gx': (_c_int, [_vp, _c_int, _c_int, _vp] + [_c_int] * 10 + [_vp, _vp]),
    'srf_route_sdr_gw': (_c_int, [_vp, _c_int, _c_int, _vp] + [_c_int] * 11 + [_vp, _vp, _vp]),
    'srf_route_sdr_pose_n': (_c_int, [_ranges] + [_c_int] * 10 + [_vp]),
    'srf_route_sdr_recur_fwd_n': (_c_int, [_ranges] + [_c_int] * 8 + [_vp]),
    'srf_route_sdr_recur_bwd_n': (_c_int, [_ranges] + [_c_int] * 8 + [_vp]),
    'srf_route_sdr_gx_n': (_c_int, [_ranges] + [_c_int] * 9 + [_vp]),
    'srf_route_sdr_gw_n': (_c_int, [_ranges] + [_c_int] * 9 + [_vp]),
    'srf_route_sdr_gx_gw_n': (_c_int, [_ranges] + [_c_int] * 9 + [_vp]),
    'srf_route_sdr_gx_gw_fact_n': (_c_int, [_ranges] + [_c_int] * 10 + [_vp]),
    'srf_cnnfe_out_dims': (_c_int, [_c_int, _c_int, ctypes.POINTER(_c_int), ctypes.POINTER(_c_int)]),
    'srf_cnnfe_saved_bytes': (_c_size, [_c_int] * 4),
    'srf_cnnfe_fwd_workspace': (_c_size, [_c_int] * 4),
    'srf_cnnfe_bwd_workspace': (_c_size, [_c_int] * 4),
    'srf_cnnfe_fwd': (_c_int, [_vp, _vp] + [_c_int] * 4 + [_vp] * 16 + [_c_int, ctypes.c_float, ctypes.c_ulonglong,
                                                                       _vp, _vp, _c_size, _vp, _c_size, _vp]),
    'srf_cnnfe_bwd': (_c_int, [_vp, _vp] + [_c_int] * 4 + [_vp] * 4 + [ctypes.c_float, ctypes.c_ulonglong]
                      + [_vp] * 15 + [_c_size, _vp]),
    'srf_cnnfe_bwd_parts': (_c_int, [_c_int, _vp, _vp] + [_c_int] * 4 + [_vp] * 4 + [ctypes.c_float, ctypes.c_ulonglong]
                            + [_vp] * 15 + [_c_size, _vp]),
    'srf_primary_caps_saved_bytes': (_c_size, [_c_int] * 4),
    'srf_primary_caps_bwd_workspace': (_c_size, [_c_int] * 5),
    'srf_primary_caps_fwd': (_c_int, [_vp, _vp] + [_c_int] * 5 + [_vp] * 8 + [_c_int, ctypes.c_float, ctypes.c_float,
                                                                           ctypes.c_ulonglong, _vp, _vp, _c_size, _vp]),
    'srf_primary_caps_bwd': (_c_int, [_vp, _vp] + [_c_int] * 5 + [_vp] * 5 + [_c_int, ctypes.c_float, ctypes.c_float,
                                                                           ctypes.c_ulonglong] + [_vp] * 12
                             + [_c_size, _vp]),
    'srf_primary_caps_fwd_ex': (_c_int, [_vp, _vp] + [_c_int] * 5 + [_vp] * 8
                                + [_c_int, ctypes.c_float, ctypes.c_float, ctypes.c_ulonglong, ctypes.c_float, _c_int,
                                   _vp, _vp, _c_size, _vp]),
    'srf_primary_caps_bwd_ex': (_c_int, [_vp, _vp] + [_c_int] * 5 + [_vp] * 5
                                + [_c_int, ctypes.c_float, ctypes.c_float, ctypes.c_ulonglong, ctypes.c_float]
                                + [_vp] * 12 + [_c_size, _vp]),
    'srf_capsnorm_bwd_workspace': (_c_size, [_c_int] * 3),
    'srf_capsnorm_fwd': (_c_int, [_vp, _c_int, _c_int, _vp, _vp, _c_int, ctypes.c_float, ctypes.c_ulonglong, _c_int,
                                  _vp, _vp, _vp]),
    'srf_capsnorm_bwd': (_c_int, [_vp, _c_int, _c_int, _vp, _vp, _c_int, ctypes.c_float, ctypes.c_ulonglong, _c_int]
                         + [_vp] * 6 + [_c_size, _vp]),
    'srf_capsnorm_fwd_range_n': (_c_int, [_cn_ranges] + [_c_int] * 5 + [ctypes.c_float, ctypes.c_ulonglong, _vp]),
    'srf_capsnorm_bwd_range_n': (_c_int, [_cn_ranges] + [_c_int] * 5 + [ctypes.c_float, ctypes.c_ulonglong, _vp]),
    'srf_capsnorm_fwd_range': (_c_int, [_vp] + [_c_int] * 5 + [_vp, _vp, _c_int, ctypes.c_float, ctypes.c_ulonglong,
                                                             _c_int, _vp, _vp, _vp]),
    'srf_capsnorm_bwd_range': (_c_int, [_vp] + [_c_int] * 5 + [_vp, _vp, _c_int, ctypes.c_float, ctypes.c_ulonglong,
                                                             _c_int, _vp, _vp, _vp, _vp, _vp]),
    'srf_capsnorm_params_workspace': (_c_size, [_c_int] * 2),
    'srf_capsnorm_bwd_params': (_c_int, [_vp, _c_int, _c_int, _vp, _vp, _vp, _c_size, _vp]),
    'srf_caps_head_fwd': (_c_int, [_vp, _c_int, _c_int, _c_int] + [_vp] * 4 + [_c_int, ctypes.c_float,
                                                                              ctypes.c_ulonglong, _c_int]
                          + [_vp] * 4),
    'srf_caps_head_fwd_ex': (_c_int, [_vp, _c_int, _c_int, _c_int] + [_vp] * 4
                             + [_c_int, ctypes.c_float, ctypes.c_ulonglong, _c_int, ctypes.c_float] + [_vp] * 4),
    'srf_caps_head_bwd': (_c_int, [_vp, _c_int, _c_int, _c_int] + [_vp] * 3 + [_c_int, ctypes.c_float,
                                                                              ctypes.c_ulonglong, _c_int]
                          + [_vp] * 9 + [_c_size, _vp]),
    'srf_ctc_workspace': (_c_size, [_c_int] * 4),
    'srf_ctc_loss': (_c_int, [_vp] * 4 + [_c_int] * 5 + [ctypes.c_float, _vp, _vp, _vp, _c_size, _vp]),
    'srf_adam_step': (_c_int, [_vp, _vp, _vp, _vp, _c_size, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                               ctypes.c_float, _vp]),
}

# include/srf_prof.h: diagnostics (bench.py's kernel timing), not the product ABI.
_PROF_SIGNATURES = {
    'srf_route_dr_set_timing_events': (_c_int, [_vp, _vp, _c_int]),
}


class SrfError(RuntimeError):
    pass


_lib = None


def lib():
    """Load (once) and return the bound library; raises if it is not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f'{LIB_PATH} is missing: build it with `make -C srf_amd/csrc` '
                              '(or __graft_entry__.build()); there is no fallback path')
        # torch must be imported first so that its HIP runtime (same SONAME as
        # /opt/rocm's) is the one this library binds to.
        import torch  # noqa: F401
        h = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in list(_SIGNATURES.items()) + list(_PROF_SIGNATURES.items()):
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _lib = h
    return _lib


def exported_symbols():
    return list(_SIGNATURES)


def prof_symbols():
    return list(_PROF_SIGNATURES)


def check(rc, what):
    if rc != 0:
        msg = lib().srf_last_error().decode(errors='replace')
        raise SrfError(f'{what} failed (rc={rc}): {msg}')
