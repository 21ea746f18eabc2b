"""ctypes binding of libmtaz.so (include/mtaz.h).

The product path has no fallback: if the HIP library is missing or fails to load,
every entry point raises MtazLibraryError.
"""
import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int32, c_int64, c_size_t, c_uint8, c_uint16, c_uint32, c_uint64, c_void_p

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('MTAZ_LIB', os.path.join(HERE, 'libmtaz.so'))
CODEC_PATH = os.path.join(HERE, 'data', 'moves_dict.json')

E_FAIL, E_ILLEGAL, E_TERMINATED, E_DEVICE, E_CAPACITY = -1, -2, -3, -4, -5
RF_DOUBLE_STEP, RF_PROMO_ALL, RF_INSUFFICIENT, RF_FIVEFOLD, RF_SEVENTYFIVE = 0x1, 0x2, 0x4, 0x8, 0x10
RF_DEFAULT = RF_PROMO_ALL | RF_INSUFFICIENT | RF_FIVEFOLD | RF_SEVENTYFIVE
KMAX = 256

P_u32, P_i32, P_u16, P_u8, P_f32, P_f64, P_i64 = (POINTER(c_uint32), POINTER(c_int32), POINTER(c_uint16),
                                                  POINTER(c_uint8), POINTER(c_float), POINTER(c_double), POINTER(c_int64))

# name -> (restype, argtypes); every symbol declared in include/mtaz.h
SIGNATURES = {
    'mtaz_abi_version': (c_int, []),
    'mtaz_version': (c_char_p, []),
    'mtaz_last_error': (c_char_p, []),
    'mtaz_load_codec': (c_int, [c_char_p]),
    'mtaz_pos_from_fen': (c_int, [c_char_p, P_u32]),
    'mtaz_pos_to_fen': (c_int, [P_u32, c_char_p, c_int]),
    'mtaz_pos_legal': (c_int, [P_u32, c_uint32, P_u16, c_int]),
    'mtaz_pos_outcome': (c_int, [P_u32, c_uint32, c_int, c_int]),
    'mtaz_pos_step': (c_int, [P_u32, c_int, c_uint32, P_u32]),
    'mtaz_pos_zeroing': (c_int, [P_u32, c_int]),
    'mtaz_pos_encode': (c_int, [P_u32, P_u8, P_f32]),
    'mtaz_rng_state_size': (c_size_t, []),
    'mtaz_rng_seed': (None, [c_void_p, c_uint32]),
    'mtaz_rng_double': (c_double, [c_void_p]),
    'mtaz_rng_dirichlet': (None, [c_void_p, c_double, c_int, P_f64]),
    'mtaz_rng_choice_p': (c_int64, [c_void_p, P_f64, c_int]),
    'mtaz_rng_randint': (c_int64, [c_void_p, c_int64]),
    'mtaz_rng_dirichlet_device': (c_int, [c_int, P_u32, P_i32, c_int, c_int, c_double, P_f64, P_f64]),
    'mtaz_legal_batch': (c_int, [c_int, c_void_p, c_int, c_uint32, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    'mtaz_encode_batch': (c_int, [c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    'mtaz_replay_put': (c_int, [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                  c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    'mtaz_create': (c_void_p, [c_int, c_int, c_int, c_double, c_int, c_double, c_double, c_uint64, c_int, c_uint32, c_int]),
    'mtaz_destroy': (None, [c_void_p]),
    'mtaz_set_weights': (c_int, [c_void_p, POINTER(c_void_p), P_i64, c_int]),
    'mtaz_evaluate': (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    'mtaz_play': (c_int, [c_void_p, c_int, c_int]),
    'mtaz_records_counts': (c_int, [c_void_p, P_i32, P_i64, P_i64]),
    'mtaz_records_get': (c_int, [c_void_p, P_u32, P_i32, P_i32, P_u16, P_u32, P_f32, P_i32]),
    'mtaz_records_json': (c_int64, [c_int, P_i32, P_u32, P_i32, P_i32, P_u16, P_u32, P_f32, c_char_p, c_char_p,
                                    c_char_p, c_void_p, c_int64, P_i64]),
    'mtaz_repr_double': (c_int, [c_double, c_char_p, c_int]),
    'mtaz_stats': (c_int, [c_void_p, P_f64, c_int]),
    'mtaz_set_timing': (c_int, [c_void_p, c_int]),
    'mtaz_set_precision': (c_int, [c_void_p, c_int]),
    'mtaz_set_seed_base': (c_int, [c_void_p, c_uint64]),
    'mtaz_set_host_threads': (c_int, [c_void_p, c_int]),
    'mtaz_set_sync_mode': (c_int, [c_void_p, c_int]),
    'mtaz_set_defer': (c_int, [c_void_p, c_int]),
    'mtaz_set_lag_order': (c_int, [c_void_p, c_int]),
    'mtaz_set_rng_device': (c_int, [c_void_p, c_int]),
    'mtaz_set_schedule': (c_int, [c_void_p, c_int]),
    'mtaz_wave_log': (c_int, [c_void_p, P_i32, c_int]),
    'mtaz_set_net_variant': (c_int, [c_void_p, c_int]),
    'mtaz_set_pipeline': (c_int, [c_void_p, c_int]),
    'mtaz_set_memo': (c_int, [c_void_p, c_int]),
    'mtaz_set_edge_capacity': (c_int, [c_void_p, c_int64, c_int64]),
    'mtaz_set_weights_slot': (c_int, [c_void_p, c_int, POINTER(c_void_p), P_i64, c_int]),
    'mtaz_set_agent_slots': (c_int, [c_void_p, c_int, c_int]),
    'mtaz_net_time': (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, P_f32, POINTER(c_uint64)]),
    'mtaz_set_games': (c_int, [c_void_p, P_u32, P_i32, P_u8, c_int]),
    'mtaz_get_games': (c_int, [c_void_p, P_u32, P_i32, P_u8, P_i32]),
    'mtaz_clear_trees': (c_int, [c_void_p, P_i32, c_int]),
    'mtaz_move_begin': (c_int, [c_void_p, P_i32, P_i32]),
    'mtaz_set_noise': (c_int, [c_void_p, P_f64, P_i64, P_i32, c_int64]),
    'mtaz_simulate': (c_int, [c_void_p, c_int, c_int]),
    'mtaz_sim_select': (c_int, [c_void_p, c_int]),
    'mtaz_leaves_get': (c_int, [c_void_p, P_i32, P_u32, P_i32, P_i32, P_u16]),
    'mtaz_leaves_set': (c_int, [c_void_p, P_f32, P_f32, c_int]),
    'mtaz_sim_evaluate': (c_int, [c_void_p]),
    'mtaz_leaves_result': (c_int, [c_void_p, P_f32, P_f32, c_int]),
    'mtaz_sim_backup': (c_int, [c_void_p]),
    'mtaz_move_end': (c_int, [c_void_p, P_u16, P_u32, P_i32, c_int]),
    'mtaz_apply': (c_int, [c_void_p, P_i32]),
    'mtaz_tree_size': (c_int, [c_void_p, c_int, P_i32, P_i32]),
    'mtaz_tree_get': (c_int, [c_void_p, c_int, P_u32, P_u32, P_u16, P_u8, P_f64, P_u16, P_f32, P_f64, P_u32]),
    'mtaz_tree_set': (c_int, [c_void_p, c_int, c_int, P_u32, P_u32, P_u16, P_u8, P_f64, P_u16, P_f32, P_f64, P_u32]),
}


class MtazLibraryError(RuntimeError):
    pass


class MtazError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f'mtaz error {code}: {msg}')
        self.code = code


_LIB = None


def lib():
    """Load libmtaz.so once (and the action codec); raise if it is unavailable."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise MtazLibraryError(f'{LIB_PATH} not built: run `python -m minitchess_alphazero_amd.build` '
                               '(the HIP extension is required; there is no CPU fallback)')
    # torch's wheel carries its own HIP runtime under the same soname (libamdhip64.so.7) as
    # /opt/rocm's: load torch first so that the process holds ONE runtime, the one torch was built
    # against (libmtaz loaded first binds /opt/rocm's, and torch then finds no GPU)
    import torch  # noqa: F401
    try:
        L = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        raise MtazLibraryError(f'cannot load {LIB_PATH}: {e}') from e
    for name, (res, args) in SIGNATURES.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    check_fingerprint(L.mtaz_version().decode())
    if L.mtaz_load_codec(CODEC_PATH.encode()) != 0:
        raise MtazLibraryError('codec load failed: ' + L.mtaz_last_error().decode())
    _LIB = L
    return L


def check_fingerprint(version):
    """The library must be built from the sources next to it (build.py source_hash, compiled into
    mtaz_version()); raises MtazLibraryError otherwise.  Skipped only where no sources exist."""
    from . import build as _build
    if not os.path.isdir(_build.CSRC):
        return
    want = _build.source_hash()
    if not version.endswith('mtaz-src-sha256=' + want):
        raise MtazLibraryError(f'{LIB_PATH} was not built from this tree ({version}; sources {want}): run '
                               '`python -m minitchess_alphazero_amd.build`')


def check(rc):
    """Raise MtazError for negative return codes (illegal / terminated map to the
    reference's BaseException subclasses in environment.py)."""
    if rc is None or rc >= 0:
        return rc
    L = lib()
    msg = L.mtaz_last_error().decode()
    if rc == E_ILLEGAL:
        from .environment import IlegalMoveException
        raise IlegalMoveException(msg)
    if rc == E_TERMINATED:
        from .environment import TerminatedEpisodeStepException
        raise TerminatedEpisodeStepException(msg)
    raise MtazError(rc, msg)


def ptr(a, ctype):
    """numpy array -> ctypes pointer (array must stay alive during the call)."""
    return a.ctypes.data_as(POINTER(ctype))
