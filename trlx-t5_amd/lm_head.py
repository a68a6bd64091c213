"""Fused lm_head projection + logprobs on MI355X.

  lm_head_logprobs(hidden, weight, labels)
      == logprobs_from_logits(hidden @ weight.T, labels)     (modeling.py:37-41 after the
         lm_head of ppo_models.py:640 / :274 / :588), experience side (no gradient)

The [.., V] logits are never written to HBM: MFMA tiles of 256 tokens x 256 vocab (ping-pong
schedule; 128 x 128 for small N) keep them in registers and reduce each tile to a partial
(max, Σexp) per token (csrc/lmhead_rows.hip).  PPOHotPath.experience_from_hidden runs the
experience step this way.

With gradients (hidden or weight requiring grad, H in {512, 768}) the same call is the loss
side's differentiable block, accelerate_ppo_model.py:96-118 (lm_head + logprobs_from_logits +
autograd back through both): csrc/lmhead_loss.hip's forward keeps lse and E_t = Σ_v p_tv·W_v
per token, and the backward forms dh_t = g_t·(W[y_t] − E_t) and dW = Σ_t g_t·(onehot − p_t)·h_t
— no [N, V] logits or dlogits in HBM.  Two plans for dW (`plan`):
  "saved_p"    the forward also stores its bf16 P tiles (trlx_lmhead_savep_bytes: 2·N·V bytes,
               the size of bf16 logits — 0.62 GB at C2) until the backward, whose dW pass reads
               them back: 3 MFMA passes in all, the count of the reference's three GEMMs
  "recompute"  nothing of size N·V is kept; the dW pass recomputes S from h and W: 4 passes
  "auto"       saved_p when dW is needed and the P buffer can be allocated (a
               torch.cuda.OutOfMemoryError on it falls back to recompute), else recompute
"""
import torch

from . import _lib

__all__ = ["lm_head_logprobs", "PLANS"]

GRAD_HIDDEN_SIZES = (512, 768)  # hidden sizes the fused backward is built for (lmhead_loss.hip)


def _operands(hidden, weight, labels):
    H = hidden.shape[-1]
    h = hidden.reshape(-1, H)
    if h.stride(-1) != 1 or h.stride(0) % 8 or h.data_ptr() % 16:
        h = h.contiguous()
    w = weight if (weight.stride(-1) == 1 and weight.stride(0) % 8 == 0 and weight.data_ptr() % 16 == 0) \
        else weight.contiguous()
    return h, w, labels.reshape(-1).contiguous()


PLANS = ("auto", "saved_p", "recompute")


def _savep_buffer(N, H, V, dev, plan):
    """The saved-P region for this call, or None (the recompute plan)."""
    if plan == "recompute":
        return None
    nbytes = _lib.query("trlx_lmhead_savep_bytes", N, H, V)
    if plan == "saved_p":
        return torch.empty(nbytes, dtype=torch.uint8, device=dev)
    try:
        return torch.empty(nbytes, dtype=torch.uint8, device=dev)
    except torch.cuda.OutOfMemoryError:
        return None


class _LmHeadLogprobs(torch.autograd.Function):
    """lp = log_softmax(h·Wᵀ)[y] with its backward, logits never materialised."""

    @staticmethod
    def forward(ctx, hidden, weight, labels, out_dtype, plan, mask):
        h, w, y = _operands(hidden, weight, labels)
        N, H, V = h.shape[0], h.shape[1], w.shape[0]
        dev = h.device
        lp = torch.empty(N, dtype=out_dtype, device=dev)
        lse = torch.empty(N, dtype=torch.float32, device=dev)
        e = torch.empty((N, H), dtype=torch.float32, device=dev)
        # the P tiles only serve the dW pass: a frozen lm_head keeps nothing of size N·V
        saved = _savep_buffer(N, H, V, dev, plan) if ctx.needs_input_grad[1] else None
        ws = torch.empty(_lib.query("trlx_lmhead_loss_workspace_bytes", N, H, V), dtype=torch.uint8, device=dev)
        _lib.call("trlx_lmhead_logprobs_fwd_ex", h.data_ptr(), h.stride(0), w.data_ptr(), w.stride(0), N, H, V,
                  y.data_ptr(), 1, _lib.ptr(mask), lp.data_ptr(), _lib.dtype_code(lp), lse.data_ptr(), e.data_ptr(),
                  ws.data_ptr(), _lib.ptr(saved), _lib.stream_of(h))
        del ws  # the forward's partials: free once the combine has run (stream-ordered)
        # the P region rides save_for_backward, so autograd frees it with the graph's other saved
        # tensors once the backward has run (not when the last reference to lp goes); the
        # backward only reads it, so a retain_graph second backward sees the same bytes
        ctx.save_for_backward(h, w, y, lse, e, saved)
        ctx.mask = mask
        ctx.shapes = (hidden.shape, hidden.dtype, weight.shape, weight.dtype)
        return lp.view(labels.shape)

    @staticmethod
    def backward(ctx, grad_lp):
        h, w, y, lse, e, saved_p = ctx.saved_tensors
        hshape, hdt, wshape, wdt = ctx.shapes
        N, H, V = h.shape[0], h.shape[1], w.shape[0]
        dev = h.device
        need_h, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        if not (need_h or need_w):
            return None, None, None, None, None, None
        g = grad_lp.reshape(-1).contiguous()
        if g.dtype not in (torch.float32, torch.bfloat16):
            g = g.float()
        # a frozen (or tied-and-handled-elsewhere) lm_head skips the dW pass entirely; the
        # buffers come from PyTorch's stream-ordered caching allocator (no hipMalloc per call
        # in steady state), and the backward's workspace holds no forward partials
        dh = torch.empty((N, H), dtype=hdt, device=dev) if need_h else None
        dw = torch.empty((V, H), dtype=wdt, device=dev) if need_w else None
        ws = torch.empty(_lib.query("trlx_lmhead_loss_bwd_workspace_bytes", N, H, V), dtype=torch.uint8, device=dev)
        saved = saved_p if need_w else None
        _lib.call("trlx_lmhead_logprobs_bwd_ex", h.data_ptr(), h.stride(0), w.data_ptr(), w.stride(0), N, H, V,
                  y.data_ptr(), 1, _lib.ptr(ctx.mask), g.data_ptr(), _lib.dtype_code(g), lse.data_ptr(), e.data_ptr(),
                  _lib.ptr(dh), H if dh is None else dh.stride(0), _lib.dtype_code(dh if dh is not None else dw),
                  _lib.ptr(dw), _lib.dtype_code(dw if dw is not None else dh), H if dw is None else dw.stride(0),
                  ws.data_ptr(), _lib.ptr(saved), _lib.stream_of(h))
        return (dh.view(hshape) if need_h else None), (dw.view(wshape) if need_w else None), None, None, None, None


def lm_head_logprobs(hidden: torch.Tensor, weight: torch.Tensor, labels: torch.Tensor, out_dtype=None,
                     return_lse: bool = False, plan: str = "auto", mask=None):
    """hidden [..., H] bf16, weight [V, H] bf16 (nn.Linear.weight), labels [...] int64 ->
    logprobs [...] of out_dtype (default: hidden.dtype, the dtype the reference's logits —
    and so its logprobs — have).  Arithmetic: bf16 products, fp32 accumulation and
    softmax statistics; the logits are not rounded to bf16 (the reference rounds them).
    Differentiable w.r.t. hidden and weight when either requires grad: for H in
    GRAD_HIDDEN_SIZES the backward runs lmhead_loss.hip's dh / dW passes (no [.., V] logits;
    `plan`: the dW pass from the forward's saved bf16 P or recomputed, see the module doc);
    other H take hipBLASLt bf16 logits + logprobs_from_logits (the reference's structure).
    mask (optional, labels' shape, any integer / bool dtype): tokens with mask == 0 get lp = 0
    and zero gradient, and the fused path compacts them out of its MFMA passes — for a consumer
    that multiplies lp by the same mask (PPOConfig.loss: ppo_models.py:150-199), where their lp
    never matters."""
    if plan not in PLANS:
        raise ValueError(f"plan must be one of {PLANS}, not {plan!r}")
    if mask is not None:
        if tuple(mask.shape) != tuple(labels.shape):
            raise ValueError(f"mask must have labels' shape {tuple(labels.shape)}, got {tuple(mask.shape)}")
        mask = mask.to(device=labels.device, dtype=torch.int64).reshape(-1).contiguous()
    _lib.require_cuda(hidden, weight, labels)
    if hidden.dtype != torch.bfloat16 or weight.dtype != torch.bfloat16:
        raise TypeError("lm_head_logprobs takes bf16 hidden states and weight")
    if labels.dtype != torch.int64:
        raise TypeError("labels must be int64")
    H = hidden.shape[-1]
    if weight.dim() != 2 or weight.shape[1] != H:
        raise ValueError(f"weight must be [V, {H}], got {tuple(weight.shape)}")
    if tuple(labels.shape) != tuple(hidden.shape[:-1]):
        raise ValueError("labels must have hidden.shape[:-1]")
    dt = hidden.dtype if out_dtype is None else out_dtype
    if torch.is_grad_enabled() and (hidden.requires_grad or weight.requires_grad):
        if return_lse:
            raise ValueError("return_lse is for the no-grad (experience) path")
        if H not in GRAD_HIDDEN_SIZES:
            # the reference's own structure for the hidden sizes the fused backward is not built
            # for: bf16 logits by hipBLASLt (autograd), the row kernels' logprobs_from_logits
            from .modeling import logprobs_from_logits
            lp = logprobs_from_logits(torch.matmul(hidden, weight.t()), labels).to(dt)
            return lp if mask is None else lp * (mask.view(labels.shape) != 0).to(dt)
        return _LmHeadLogprobs.apply(hidden, weight, labels, dt, plan, mask)
    h, w, y = _operands(hidden, weight, labels)
    N, V = h.shape[0], w.shape[0]
    lp = torch.empty(N, dtype=dt, device=h.device)
    lse = torch.empty(N, dtype=torch.float32, device=h.device) if return_lse else None
    ws = torch.empty(_lib.query("trlx_lmhead_workspace_bytes", N, V), dtype=torch.uint8, device=h.device)
    _lib.call("trlx_lmhead_logprobs", h.data_ptr(), h.stride(0), w.data_ptr(), w.stride(0), N, H, V, y.data_ptr(), 1,
              lp.data_ptr(), _lib.dtype_code(lp), _lib.ptr(lse), ws.data_ptr(), _lib.stream_of(h))
    lp = lp.view(labels.shape)
    if mask is not None:  # the experience path: every row computed, the skipped ones zeroed
        drop = mask.view(labels.shape) == 0
        lp.masked_fill_(drop, 0.0)
        if lse is not None:
            lse.view(labels.shape).masked_fill_(drop, 0.0)
    return (lp, lse.view(labels.shape)) if return_lse else lp
