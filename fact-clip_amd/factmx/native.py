"""ctypes binding of libfactmx.so (the C ABI declared in include/factmx.h).

The product path has no CPU or eager-PyTorch fallback: importing an op that
needs the library raises ``FactmxNativeError`` when the .so is missing or was
built for another ABI, and every non-zero status from a call raises with the
library's ``fx_last_error()`` text.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FACTMX_LIB", os.path.join(_HERE, "_lib", "libfactmx.so"))
ABI_VERSION = 20

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_longlong
F = ctypes.c_float
D = ctypes.c_double
U = ctypes.c_ulonglong


class FactmxNativeError(RuntimeError):
    pass


class Operand(ctypes.Structure):
    _fields_ = [("ptr", P), ("ld", L), ("ptr1", P), ("ld1", L), ("k_split", I), ("rows0", P), ("rows1", P),
                ("pos", P), ("ld_pos", L), ("pos_cols", I), ("trans", I), ("conv_taps", I), ("conv_cin", I),
                ("conv_dil", I), ("conv_dir", I), ("seq_len", I), ("batch_stride", L), ("ones_col", I),
                ("seq_off", P), ("nseq", I)]


class GemmDesc(ctypes.Structure):
    _fields_ = [("M", I), ("N", I), ("K", I), ("batch", I), ("a", Operand), ("b", Operand), ("c", P), ("ldc", L),
                ("c_batch_stride", L), ("alpha", F), ("beta", F), ("bias", P), ("resid", P), ("ld_resid", L),
                ("resid_batch_stride", L), ("gate", P), ("ld_gate", L), ("relu", I), ("c_tap_cin", I),
                ("split_k", I), ("workspace", P), ("c_last_col", P), ("dbg_stamps", P), ("drop_p", F),
                ("drop_seed", U), ("c_last_batch_stride", L), ("b_dil_growth", I),
                ("a_dil_b1", I), ("bias_batch_stride", L)]


class MstcnParams(ctypes.Structure):
    _fields_ = [("cin", I), ("F", I), ("cout", I), ("num_layers", I), ("layernorm", I), ("in_map", I),
                ("dil0", I), ("dil_factor", I), ("w_in", P), ("b_in", P), ("w_dil", P), ("b_dil", P), ("w_pw", P), ("b_pw", P),
                ("ln_w", P), ("ln_b", P), ("w_out", P), ("b_out", P), ("dropout", F), ("seed", U),
                ("side_defer", I), ("seq_off", P), ("fused_layers", I)]


class Mstcn2Params(ctypes.Structure):
    _fields_ = [("cin", I), ("F", I), ("cout", I), ("num_layers", I), ("in_map", I), ("dil_factor", I),
                ("w_in", P), ("b_in", P), ("w_d1", P), ("b_d1", P), ("w_d2", P), ("b_d2", P), ("w_fu", P),
                ("b_fu", P), ("w_out", P), ("b_out", P), ("dropout", F), ("seed", U), ("side_defer", I),
                ("seq_off", P)]


class Mstcn2Grads(ctypes.Structure):
    _fields_ = [("w_in", P), ("b_in", P), ("w_d1", P), ("b_d1", P), ("w_d2", P), ("b_d2", P), ("w_fu", P),
                ("b_fu", P), ("w_out", P), ("b_out", P)]


class MstcnGrads(ctypes.Structure):
    _fields_ = [("w_in", P), ("b_in", P), ("w_dil", P), ("b_dil", P), ("w_pw", P), ("b_pw", P),
                ("ln_w", P), ("ln_b", P), ("w_out", P), ("b_out", P)]


_DEC_PTRS = ["sa_in_w", "sa_in_b", "sa_out_w", "sa_out_b", "ca_q_w", "ca_k_w", "ca_v_w", "ca_in_b", "ca_out_w",
             "ca_out_b", "ff1_w", "ff1_b", "ff2_w", "ff2_b", "ln_sa_w", "ln_sa_b", "ln_ca_w", "ln_ca_b", "ln_ff_w",
             "ln_ff_b"]
DECODER_LAYER_FIELDS = _DEC_PTRS
DECODER_GLOBAL_FIELDS = ["fn_w", "fn_b", "out_w", "out_b"]


class DecoderParams(ctypes.Structure):
    _fields_ = ([("A", I), ("FF", I), ("nhead", I), ("num_layers", I), ("cross", I), ("Hm", I), ("out_dim", I),
                 ("final_norm", I), ("eps", F)] + [(n, P) for n in _DEC_PTRS] + [(n, P) for n in DECODER_GLOBAL_FIELDS]
                + [("side_defer", I), ("dropout", F), ("attn_dropout", F), ("seed", U), ("mem_off", P), ("status", P),
                   ("dqpos_accumulate", I)])


class DecoderGrads(ctypes.Structure):
    _fields_ = [(n, P) for n in _DEC_PTRS] + [(n, P) for n in DECODER_GLOBAL_FIELDS]


STATUS_GRU_TIMEOUT = 1   # FX_STATUS_GRU_TIMEOUT: a BiGRU workgroup gave up waiting for a peer
STATUS_TOK_TIMEOUT = 2   # FX_STATUS_TOK_TIMEOUT: a persistent token-kernel barrier wait gave up
STATUS_X2Y_TIMEOUT = 4   # FX_STATUS_X2Y_TIMEOUT: the one-launch X2Y f2a backward's grid barrier gave up
LOSS_MAXK = 512        # FX_LOSS_MAXK: matched columns of an attention loss term
LOSS_NB = 128          # FX_LOSS_NB: row blocks per loss term
TERM_CLASS, TERM_ATTN, TERM_INFONCE = 0, 1, 2
PREC_DEFAULT, PREC_F32, PREC_BF16, PREC_F32S, PREC_F32S2 = -1, 0, 1, 2, 3   # FX_PREC_*: GEMM arithmetic


class LossTerm(ctypes.Structure):
    _fields_ = [("kind", I), ("slot", I), ("R", I), ("C", I), ("x", P), ("sr", L), ("sc", L), ("dx", P), ("dsr", L),
                ("dsc", L), ("y", P), ("rs", P), ("re", P), ("gs", P), ("ge", P), ("gl", P), ("G", I), ("axis", I),
                ("K", I), ("D", I), ("w", P), ("c_ce", F), ("c_sm", F), ("inv_temp", F), ("pad0", F), ("lse", P),
                ("lse2", P), ("colz", P), ("emb", P), ("ld_emb", L), ("text", P), ("demb", P), ("ld_demb", L),
                ("ka", P), ("kgs", P), ("kge", P), ("ksw", P)]


class VideoAttn(ctypes.Structure):
    _fields_ = [("Q", I), ("C1", I), ("T", I), ("G", I), ("clogit", P), ("ldc", L), ("attn", P), ("lda", L),
                ("seg_id", P), ("flogit", P), ("ldf", L), ("gs", P), ("ge", P), ("gl", P), ("pred_off", L)]


ABI_STRUCTS = (GemmDesc, DecoderParams, MstcnParams, LossTerm, VideoAttn, Mstcn2Params)   # fx_struct_size ids


# name -> (restype, argtypes); every fx_* symbol declared in include/factmx.h
SIGNATURES = {
    "fx_version": (I, []),
    "fx_last_error": (ctypes.c_char_p, []),
    "fx_struct_size": (L, [I]),
    "fx_gemm": (I, [ctypes.POINTER(GemmDesc), P]),
    "fx_gemm_workspace_floats": (L, [ctypes.POINTER(GemmDesc)]),
    "fx_linear_fwd": (I, [P, L, P, L, I, I, I, P, L, P, P, L, I, I, P]),
    "fx_linear_bwd_workspace_floats": (L, [I, I, I]),
    "fx_linear_bwd": (I, [P, L, P, L, P, L, P, L, I, I, I, P, L, P, L, P, I, I, P, P]),
    "fx_x2y_saved_floats": (L, [I, I, I, I, I]),
    "fx_x2y_workspace_floats": (L, [I, I, I, I, I, I, I, P, P]),
    "fx_x2y_fwd": (I, [P, L, I, I, P, L, I, P, L, I, I, P, L, I, P, P, P, P, P, P, P, P, I, I, I, P, P, F, U, P, L, P,
                       P, P, P, P]),
    "fx_x2y_bwd": (I, [P, L, I, I, I, P, L, I, I, I, P, P, P, P, I, I, I, P, P, F, U, P, P, P, L, P, P, P, P, P, P,
                       P, P, P, P, P, P, P, P, I, I, P, I, P, P]),
    "fx_decoder_saved_floats": (L, [ctypes.POINTER(DecoderParams), I, I, I, I, I]),
    "fx_decoder_workspace_floats": (L, [ctypes.POINTER(DecoderParams), I, I, I, I, I]),
    "fx_tok_gemm": (I, [P, L, I, I, I, I, P, P, P, L, I, P, P, L, P, L, P, P]),
    "fx_decoder_fwd": (I, [ctypes.POINTER(DecoderParams), P, L, I, P, L, P, L, I, I, P, L, P, L, P, P, P]),
    "fx_decoder_bwd": (I, [ctypes.POINTER(DecoderParams), ctypes.POINTER(DecoderGrads), P, L, I, P, P, L, I, I, P, L,
                           P, L, P, L, P, P, L, P, L, P, P, P]),
    "fx_mstcn_saved_floats": (L, [ctypes.POINTER(MstcnParams), I]),
    "fx_side_stream": (P, []),
    "fx_side_join": (I, [P]),
    "fx_mstcn_workspace_floats": (L, [ctypes.POINTER(MstcnParams), I]),
    "fx_mstcn_fwd": (I, [ctypes.POINTER(MstcnParams), P, L, I, I, P, L, P, P, P]),
    "fx_mstcn_bwd": (I, [ctypes.POINTER(MstcnParams), ctypes.POINTER(MstcnGrads), P, L, I, I, P, L, P, L, P, P, P]),
    "fx_mstcn2_saved_floats": (L, [ctypes.POINTER(Mstcn2Params), I]),
    "fx_mstcn2_workspace_floats": (L, [ctypes.POINTER(Mstcn2Params), I]),
    "fx_mstcn2_fwd": (I, [ctypes.POINTER(Mstcn2Params), P, L, I, I, P, L, P, P, P]),
    "fx_mstcn2_bwd": (I, [ctypes.POINTER(Mstcn2Params), ctypes.POINTER(Mstcn2Grads), P, L, I, I, P, L, P, L, P, P, P]),
    "fx_layernorm_fwd": (I, [P, L, P, L, P, P, F, I, I, I, P, L, P, L, P, P]),
    "fx_layernorm_bwd_workspace_floats": (L, [I, I]),
    "fx_layernorm_bwd": (I, [P, L, P, L, P, L, P, P, I, I, I, P, L, P, P, P, P]),
    "fx_softmax_rows": (I, [P, L, I, I, F, P, L, P]),
    "fx_softmax_rows_bwd": (I, [P, L, P, L, P, L, I, I, F, P, L, P]),
    "fx_process_feature_fwd": (I, [P, L, I, I, I, P, L, P, L, P]),
    "fx_process_feature_bwd": (I, [P, L, P, L, P, L, I, I, I, P, L, P]),
    "fx_l2norm_fwd": (I, [P, L, I, I, P, L, P, P]),
    "fx_l2norm_bwd": (I, [P, L, P, P, L, I, I, P, L, P]),
    "fx_relu_bwd": (I, [P, L, P, L, I, I, P, L, P]),
    "fx_add": (I, [P, L, P, L, I, I, P, L, I, P]),
    "fx_mha_t_workspace_floats": (L, [I, I, I, I, I]),
    "fx_mha_t_fwd": (I, [P, L, P, L, P, L, I, I, I, I, I, F, P, L, P, P, P]),
    "fx_mha_t_bwd": (I, [P, L, P, L, P, L, P, L, P, L, P, I, I, I, I, I, F, P, L, P, L, P, L, P, P]),
    "fx_mha_core_workspace_floats": (L, [I, I, I, I]),
    "fx_mha_core_fwd": (I, [P, L, P, L, P, L, I, I, I, I, F, U, P, P, L, P, P]),
    "fx_mha_core_bwd": (I, [P, L, P, L, P, L, P, P, L, I, I, I, I, F, U, P, L, P, L, P, L, P, P]),
    "fx_dropout": (I, [P, L, I, I, L, L, F, U, P, L, P]),
    "fx_gru_saved_floats": (L, [I, I]),
    "fx_gru_workspace_floats": (L, [I, I, I, I]),
    "fx_gru_bidir_fwd": (I, [P, L, I, I, P, I, I, P, P, P, P, P, P, P, P, P, L, I, P, P, P, I, P]),
    "fx_gru_bidir_bwd": (I, [P, L, I, I, P, I, I, P, P, P, P, P, P, L, P, L, P, L, P, P, P, P, P, P, P, P, P, P, I,
                             P]),
    "fx_segments_from_probs": (I, [P, L, I, I, I, I, P, P, P, P, P, P, P]),
    "fx_segments_globalize": (I, [I, I, P, P, P, P, P, P, P, P, P]),
    "fx_seg_mean_fwd": (I, [P, L, P, P, I, I, P, L, P]),
    "fx_seg_mean_bwd": (I, [P, L, P, P, P, I, I, P, L, I, P]),
    "fx_seg_sum_rows": (I, [P, L, P, P, I, I, P, L, I, P]),
    "fx_grad_norm_workspace_floats": (L, []),
    "fx_grad_norm": (I, [P, L, P, P, P]),
    "fx_clip_grad_scale": (I, [P, L, P, F, P]),
    "fx_adam_step": (I, [P, P, P, P, L, L, F, F, F, F, F, F, P, P, P]),
    "fx_adam_step_checked": (I, [P, P, P, P, L, L, F, F, F, F, F, F, P, P, P, P]),
    "fx_loss_workspace_floats": (L, []),
    "fx_class_loss_fwd": (I, [P, L, L, I, I, P, P, P, F, F, P, P, P, P]),
    "fx_class_loss_bwd": (I, [P, L, L, I, I, P, P, P, P, F, F, P, P, P]),
    "fx_attn_loss_fwd": (I, [P, L, L, I, I, I, P, P, P, P, I, I, F, F, P, P, P, P, P, P]),
    "fx_attn_loss_bwd": (I, [P, L, L, I, I, I, P, P, P, P, I, I, P, P, P, F, F, P, P, L, L, P]),
    "fx_loss_terms_workspace_floats": (L, [I]),
    "fx_loss_terms_fwd": (I, [P, P, I, P, I, P, P, P]),
    "fx_loss_terms_bwd": (I, [P, P, I, P, I, P, P, P]),
    "fx_match_cost": (I, [P, P, I, F, F, I, P, P]),
    "fx_eval_pred": (I, [P, P, I, F, P, P]),
    "fx_set_stream_precision": (I, [P, I]),
    "fx_get_stream_precision": (I, [P]),
    "fx_stream_precision_explicit": (I, [P]),
    "fx_set_default_precision": (I, [I]),
    "fx_get_default_precision": (I, []),
    "fx_prof_enable": (I, [I, I]),
    "fx_prof_collect": (I, [I, ctypes.POINTER(D), ctypes.POINTER(D), ctypes.POINTER(D), ctypes.POINTER(I)]),
    "fx_prof_collect_kernels": (I, [I, ctypes.POINTER(D), ctypes.POINTER(I), ctypes.POINTER(I)]),
    "fx_prof_disable": (None, []),
    "fx_debug_set_spin": (I, [I, I]),
}

_lib = None


def load(path=None):
    """Load and type the library once.  Raises FactmxNativeError if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or LIB_PATH
    if not os.path.exists(path):
        raise FactmxNativeError(
            f"libfactmx.so not found at {path}: build it with `make -C fact-clip_amd/csrc` "
            "(or __graft_entry__.build()); factmx has no CPU/eager fallback")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.fx_version()
    if v != ABI_VERSION:
        raise FactmxNativeError(f"libfactmx ABI {v} != expected {ABI_VERSION}")
    for i, st in enumerate(ABI_STRUCTS):
        if lib.fx_struct_size(i) != ctypes.sizeof(st):
            raise FactmxNativeError(f"{st.__name__}: C size {lib.fx_struct_size(i)} != ctypes {ctypes.sizeof(st)}")
    _lib = lib
    return lib


# ctypes array TYPES by (element type, length).  ctypes' own cache of ``c_int * n`` holds its types
# weakly, so a type made per call dies after it -- and every type object sits in a reference cycle:
# per-step cyclic garbage that only a full (gen-2) collection frees, a ~60 ms host stall every few
# dozen training steps (round 4, tools/r04_gc_cycles.py).  Keeping the types here makes the per-call
# arrays plain refcounted objects.
_ARRAY_TYPES = {}


def array_type(ctype, n):
    t = _ARRAY_TYPES.get((ctype, n))
    if t is None:
        t = _ARRAY_TYPES[(ctype, n)] = ctype * n
    return t


def float_array(vals):
    """Host float32 array for the C ABI (None -> NULL)."""
    if vals is None:
        return None
    return array_type(ctypes.c_float, max(len(vals), 1))(*[float(v) for v in vals])


def int_array(vals):
    """Host int32 array for the C ABI's prefix-offset arguments (None -> NULL)."""
    if vals is None:
        return None
    return array_type(ctypes.c_int, len(vals))(*[int(v) for v in vals])


def check(status, what):
    if status != 0:
        msg = load().fx_last_error().decode(errors="replace")
        raise FactmxNativeError(f"{what} failed ({status}): {msg}")


def stream():
    return torch.cuda.current_stream().cuda_stream


def ptr(t):
    """Raw device pointer of a tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


def ld(t):
    """Row stride of a 2-D row-major (possibly column-sliced) tensor."""
    if t is None:
        return 0
    assert t.dim() == 2 and (t.stride(1) == 1 or t.shape[1] == 1), f"need unit column stride, got {t.stride()}"
    return t.stride(0)
