"""ctypes binding of libottohip.so (the C-ABI in include/ottohip.h).

There is no CPU fallback: if the library is missing or no GPU is present, every compute
entry point raises. Device buffers are torch tensors (plumbing only)."""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# OTTOHIP_LIB: another build of the same C-ABI (development A/B runs); default the in-tree library
LIB_PATH = os.environ.get("OTTOHIP_LIB") or os.path.join(_HERE, "libottohip.so")

OTTOHIP_ELIMIT = -5


class OttoHipError(RuntimeError):
    def __init__(self, rc: int, msg: str):
        super().__init__(f"ottohip error {rc}: {msg}")
        self.rc = rc


class Rule(ctypes.Structure):
    _fields_ = [("this_type", ctypes.c_int32), ("next_type_mask", ctypes.c_uint32), ("max_abs_dt", ctypes.c_int32)]


class Events(ctypes.Structure):
    _fields_ = [
        ("session_offsets", ctypes.c_void_p), ("n_sessions", ctypes.c_int64),
        ("aid", ctypes.c_void_p), ("ts", ctypes.c_void_p), ("type", ctypes.c_void_p),
        ("n_events", ctypes.c_int64),
        ("file_session_bounds", ctypes.c_void_p), ("n_files", ctypes.c_int32),
    ]


class CovisParams(ctypes.Structure):
    _fields_ = [("min_dt", ctypes.c_int32), ("max_dt", ctypes.c_int32), ("n_items", ctypes.c_int32),
                ("dedup", ctypes.c_int32), ("sym", ctypes.c_int32)]


class RuleStats(ctypes.Structure):
    _fields_ = [("n_rows", ctypes.c_int64), ("n_pairs", ctypes.c_int64), ("file_rows", ctypes.c_int64),
                ("file_rows_ge2", ctypes.c_int64)]


class FileOpts(ctypes.Structure):
    _fields_ = [("rule", ctypes.c_int32), ("lo_file", ctypes.c_int32), ("hi_file", ctypes.c_int32),
                ("n_files", ctypes.c_int32), ("lo_key", ctypes.c_uint64), ("hi_key", ctypes.c_uint64),
                ("file_rows", ctypes.c_void_p), ("file_rows_ge2", ctypes.c_void_p), ("keep_words", ctypes.c_int32)]


class PartOpts(ctypes.Structure):
    _fields_ = [("n_files", ctypes.c_int32), ("n_parts", ctypes.c_int32), ("first_part", ctypes.c_void_p),
                ("n_cuts", ctypes.c_int32), ("cut_file", ctypes.c_void_p), ("cut_key", ctypes.c_void_p)]


class MergeParams(ctypes.Structure):
    _fields_ = [("click_rule", ctypes.c_int32), ("min_count_in_part", ctypes.c_int32), ("min_count", ctypes.c_int32),
                ("max_rows", ctypes.c_int64), ("filter_rows", ctypes.c_int64), ("max_rows_groupby", ctypes.c_int64)]


# name -> (restype, argtypes); the exported symbol set of include/ottohip.h
_VP, _I32, _I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
SIGNATURES = {
    "ottohip_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_VP)]),
    "ottohip_ctx_destroy": (None, [_VP]),
    "ottohip_last_error": (ctypes.c_char_p, []),
    "ottohip_ctx_trim": (ctypes.c_int, [_VP]),
    "ottohip_ctx_set_timing": (ctypes.c_int, [_VP, ctypes.c_int]),
    "ottohip_ctx_timing": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                          ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_double)]),
    "ottohip_covis_count": (ctypes.c_int, [_VP, ctypes.POINTER(Events), ctypes.POINTER(Rule), ctypes.c_int,
                                           ctypes.POINTER(CovisParams), ctypes.POINTER(_VP), _VP]),
    "ottohip_covis_count_opts": (ctypes.c_int, [_VP, ctypes.POINTER(Events), ctypes.POINTER(Rule), ctypes.c_int,
                                                ctypes.POINTER(CovisParams), ctypes.POINTER(FileOpts),
                                                ctypes.POINTER(_VP), _VP]),
    "ottohip_covis_count_parts": (ctypes.c_int, [_VP, _VP, _VP, ctypes.c_int, ctypes.POINTER(CovisParams),
                                                 ctypes.POINTER(PartOpts), ctypes.POINTER(_VP), _VP]),
    "ottohip_table_count_parts": (ctypes.c_int, [_VP, _VP, ctypes.c_int, ctypes.POINTER(PartOpts), ctypes.POINTER(_VP),
                                                  _VP]),
    "ottohip_table_part_heads": (ctypes.c_int, [_VP, _VP, ctypes.c_int, ctypes.c_int, _I32, _I64, _VP, _I64,
                                                ctypes.POINTER(_I64), _VP]),
    "ottohip_table_keys_at": (ctypes.c_int, [_VP, _VP, ctypes.c_int, ctypes.c_int, _VP, ctypes.c_int, _VP, _VP]),
    "ottohip_table_keys_at_parts": (ctypes.c_int, [_VP, _VP, ctypes.c_int, ctypes.c_int, _VP, _VP, _VP, _VP]),
    "ottohip_table_stats": (ctypes.c_int, [_VP, ctypes.c_int, ctypes.POINTER(RuleStats)]),
    "ottohip_table_copy": (ctypes.c_int, [_VP, ctypes.c_int, _VP, _VP, _VP, _VP, _VP]),
    "ottohip_table_free": (None, [_VP]),
    "ottohip_table_finalize": (ctypes.c_int, [_VP, _VP, ctypes.c_int, ctypes.POINTER(MergeParams), _VP, _VP, _VP,
                                              ctypes.POINTER(_I64), _VP]),
    "ottohip_table_set_file_stats": (ctypes.c_int, [_VP, ctypes.c_int, _I64, _I64]),
    "ottohip_concat_tables": (ctypes.c_int, [_VP, ctypes.c_int, _VP, _VP, _VP, _VP, _I32, ctypes.POINTER(MergeParams),
                                             _I64, ctypes.c_int, _VP, _VP, _VP, ctypes.POINTER(_I64), _VP]),
    "ottohip_table_digest": (ctypes.c_int, [_VP, _VP, ctypes.c_int, _VP, _VP]),
    "ottohip_run_hist": (ctypes.c_int, [_VP, _VP, _I64, _I64, ctypes.c_int, ctypes.c_uint32, _I64, _VP, _VP]),
    "ottohip_events_csr": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _I64, _I64, _VP, _VP, _VP, _VP, _VP,
                                          ctypes.POINTER(_I64), ctypes.POINTER(ctypes.c_int), _VP]),
    "ottohip_events_csr_files": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, ctypes.c_int, _VP, _VP, _VP, _VP, _VP, _VP,
                                                _VP, ctypes.POINTER(ctypes.c_int), _VP]),
    "ottohip_topk_per_aid": (ctypes.c_int, [_VP, _VP, _VP, _VP, _I64, _I32, ctypes.c_int] + [_VP] * 7 +
                             [ctypes.POINTER(_I64), _VP]),
    "ottohip_lists_build": (ctypes.c_int, [_VP, _VP, _VP, _VP, _I64, _I32, _VP, _VP, _VP, _VP]),
    "ottohip_candidates_generate": (ctypes.c_int, [_VP, _VP, _I64, _VP, _VP, _VP, _VP, _VP, ctypes.POINTER(_VP), _VP]),
    "ottohip_candidates_info": (ctypes.c_int, [_VP, ctypes.POINTER(_I64), ctypes.POINTER(_I64)]),
    "ottohip_candidates_view": (ctypes.c_int, [_VP, ctypes.POINTER(_VP), ctypes.POINTER(_VP), ctypes.POINTER(_VP),
                                               ctypes.POINTER(_VP)]),
    "ottohip_candidates_copy": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _VP]),
    "ottohip_candidates_free": (None, [_VP]),
    "ottohip_labels_csr": (ctypes.c_int, [_VP, _VP, _I64, _VP, _VP, _VP, _I64, _VP, _VP, ctypes.POINTER(_I64), _VP]),
    "ottohip_candidates_recall": (ctypes.c_int, [_VP, _VP, _VP, _VP, ctypes.c_uint32, ctypes.c_int,
                                                 ctypes.POINTER(_I64), _VP]),
    "ottohip_session_embeddings": (ctypes.c_int, [_VP, _VP, _I64, _VP, _VP, _VP, _VP, _I32, _VP, ctypes.c_int, _VP, _VP]),
    "ottohip_kmeans_step": (ctypes.c_int, [_VP, _VP, _I64, ctypes.c_int, _VP, ctypes.c_int, _VP,
                                           ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), _VP]),
    "ottohip_kmeans_assign": (ctypes.c_int, [_VP, _VP, _I64, ctypes.c_int, _VP, ctypes.c_int, _VP,
                                             ctypes.POINTER(ctypes.c_double), _VP]),
    "ottohip_kmeans_partial": (ctypes.c_int, [_VP, _VP, _I64, ctypes.c_int, _VP, ctypes.c_int, _VP, _VP, _VP,
                                              ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_I64), _VP]),
    "ottohip_kmeans_update": (ctypes.c_int, [_VP, _VP, _VP, _VP, ctypes.c_int, ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_double), _VP]),
    "ottohip_rs_create": (ctypes.c_int, [ctypes.c_uint32, ctypes.POINTER(_VP)]),
    "ottohip_rs_permutation_head": (ctypes.c_int, [_VP, _I64, ctypes.c_int, _VP]),
    "ottohip_rs_destroy": (None, [_VP]),
    "ottohip_kmeans_lloyd_iter": (ctypes.c_int, [_VP, _VP, _I64, ctypes.c_int, _VP, ctypes.c_int, _VP, _VP, _VP,
                                                 ctypes.POINTER(ctypes.c_double), _VP]),
    "ottohip_kmeans_attach_half": (ctypes.c_int, [_VP, _VP, _I64, ctypes.c_int, _VP]),
    "ottohip_kmeans_detach_half": (ctypes.c_int, [_VP]),
    "ottohip_kmeans_lloyd_steps": (ctypes.c_int, [_VP, _VP, _I64, ctypes.c_int, _VP, ctypes.c_int, _VP, _VP, _VP,
                                                  ctypes.c_int, ctypes.c_double, ctypes.POINTER(ctypes.c_double), _VP]),
    "ottohip_kmeans_lloyd_steps_pair": (ctypes.c_int, [_VP, _VP, _I64, ctypes.c_int, _VP, ctypes.c_int, _VP, _VP,
                                                       _VP, _VP, ctypes.c_double, ctypes.POINTER(ctypes.c_double),
                                                       _VP]),
    "ottohip_kmeans_lloyd_steps_multi": (ctypes.c_int, [_VP, _VP, _I64, ctypes.c_int, _VP, ctypes.c_int, _VP, _VP,
                                                        _VP, _VP, ctypes.c_int, ctypes.c_double,
                                                        ctypes.POINTER(ctypes.c_double), _VP]),
    "ottohip_kmeans_farthest": (ctypes.c_int, [_VP, _VP, _I64, ctypes.c_int, _VP, _VP, ctypes.c_int, _VP, _VP, _VP]),
    "ottohip_kmeans_relocate": (ctypes.c_int, [_VP, _VP, _VP, ctypes.c_int, ctypes.c_int, _VP, _VP, ctypes.c_int, _VP]),
    "ottohip_kmeans_inertia": (ctypes.c_int, [_VP, _VP, _I64, ctypes.c_int, _VP, _VP, ctypes.POINTER(ctypes.c_double),
                                              _VP]),
    "ottohip_col_sums": (ctypes.c_int, [_VP, _VP, _I64, ctypes.c_int, _VP, _VP, _VP, _VP]),
    "ottohip_center_rows": (ctypes.c_int, [_VP, _VP, _I64, ctypes.c_int, _VP, _VP, _VP]),
    "ottohip_popularity_ranks": (ctypes.c_int, [_VP, _VP, _I64, _VP, _VP, _VP, _VP, _I32, _I32, _I32, ctypes.c_int,
                                                ctypes.POINTER(_VP), ctypes.POINTER(_I64), _VP]),
    "ottohip_pop_counts": (ctypes.c_int, [_VP, _VP, _I64, _VP, _VP, _VP, _VP, _I32, _I32, _I32, _VP, _VP]),
    "ottohip_popularity_from_counts": (ctypes.c_int, [_VP, _VP, _I32, _I32, ctypes.c_int, ctypes.POINTER(_VP),
                                                      ctypes.POINTER(_I64), _VP]),
    "ottohip_pop_copy": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP]),
    "ottohip_pop_free": (None, [_VP]),
    "ottohip_session_item_similarity": (ctypes.c_int, [_VP, _VP, _I64, _VP, _VP, _VP, _VP, _I32, _VP, ctypes.c_int,
                                                       _VP, _VP, _VP]),
    "ottohip_owner_of": (ctypes.c_int, [_I32, ctypes.c_int]),
    "ottohip_table_pack_by_owner": (ctypes.c_int, [_VP, _VP, ctypes.c_int, _VP, ctypes.POINTER(_I64), _VP]),
    "ottohip_table_from_records": (ctypes.c_int, [_VP, _VP, _I64, ctypes.c_int, _I32, ctypes.POINTER(RuleStats),
                                                  ctypes.POINTER(_VP), _VP]),
    "ottohip_covis_emit": (ctypes.c_int, [_VP, ctypes.POINTER(Events), ctypes.POINTER(Rule), ctypes.c_int,
                                          ctypes.POINTER(CovisParams), _VP, _I32, ctypes.c_int, ctypes.POINTER(_VP),
                                          ctypes.POINTER(_I64), ctypes.POINTER(_I64), _VP]),
    "ottohip_emit_write": (ctypes.c_int, [_VP, _VP, _VP, _VP]),
    "ottohip_emit_free": (None, [_VP]),
    "ottohip_covis_reduce_received": (ctypes.c_int, [_VP, ctypes.POINTER(Rule), ctypes.c_int, ctypes.POINTER(CovisParams),
                                                     _I32, _VP, _I64, _VP, _I64, ctypes.POINTER(_VP), _VP]),
    "ottohip_covis_reduce_received_opts": (ctypes.c_int, [_VP, ctypes.POINTER(Rule), ctypes.c_int,
                                                          ctypes.POINTER(CovisParams), _I32, _VP, _I64, _VP, _I64,
                                                          ctypes.POINTER(FileOpts), ctypes.POINTER(_VP), _VP]),
    "ottohip_knn_index_create": (ctypes.c_int, [_VP, _VP, _I64, ctypes.c_int, ctypes.POINTER(_VP), _VP]),
    "ottohip_knn_topk": (ctypes.c_int, [_VP, _VP, _VP, _I64, ctypes.c_int, _VP, _VP, _VP]),
    "ottohip_knn_index_free": (None, [_VP]),
    "ottohip_test_exclusive_scan_u32": (ctypes.c_int, [_VP, _VP, _VP, _I64, ctypes.POINTER(ctypes.c_uint64), _VP]),
    "ottohip_test_radix_sort_pairs": (ctypes.c_int, [_VP, _VP, _VP, _I64, ctypes.c_int, _VP]),
    "ottohip_test_lanes": (ctypes.c_int, [_VP, _VP, _VP]),
}

_LIB = None


def load() -> ctypes.CDLL:
    """Load libottohip.so (raises if it was not built: no fallback path exists)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with __graft_entry__.build()")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("OTTOHIP_LIB") and not hasattr(lib, name):
                continue  # an older build under A/B (development runs): entry points it lacks stay unbound
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = lib
    return _LIB


def check(rc: int):
    if rc != 0:
        raise OttoHipError(rc, load().ottohip_last_error().decode(errors="replace"))


def require_gpu():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("otto-recommender_amd needs a ROCm GPU (MI355X); no CPU fallback exists")


def stream_handle(stream=None) -> int:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def ptr(t) -> int:
    return 0 if t is None else int(t.data_ptr())


class Context:
    """One ottohip context (device workspace + timing) per device."""

    def __init__(self, device: int = 0):
        require_gpu()
        import torch
        torch.cuda.set_device(device)
        self.device = device
        self.h = ctypes.c_void_p()
        check(load().ottohip_ctx_create(device, ctypes.byref(self.h)))

    def close(self):
        if self.h:
            load().ottohip_ctx_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def trim(self):
        """Return the workspace and spare table buffers to the device (ottohip_ctx_trim)."""
        check(load().ottohip_ctx_trim(self.h))

    def set_timing(self, on: bool):
        check(load().ottohip_ctx_set_timing(self.h, 1 if on else 0))

    def timings(self) -> list:
        lib = load()
        n = lib.ottohip_ctx_timing(self.h, -1, None, None, None)
        out = []
        for i in range(max(n, 0)):
            name = ctypes.c_char_p(); ms = ctypes.c_float(); b = ctypes.c_double()
            check(lib.ottohip_ctx_timing(self.h, i, ctypes.byref(name), ctypes.byref(ms), ctypes.byref(b)))
            out.append((name.value.decode(), float(ms.value), float(b.value)))
        return out


_CTX = {}


_LANE_CTX: dict = {}


def lane_context(device: int, lane: int) -> Context:
    """A further context of `device` for work issued from another host thread on its own stream (KMeans run
    lanes): its own workspace and per-call state; cached per (device, lane)."""
    key = (int(device), int(lane))
    if key not in _LANE_CTX:
        _LANE_CTX[key] = Context(int(device))
    return _LANE_CTX[key]


def context(device: int | None = None) -> Context:
    import torch
    d = torch.cuda.current_device() if device is None else device
    if d not in _CTX:
        _CTX[d] = Context(d)
    return _CTX[d]
