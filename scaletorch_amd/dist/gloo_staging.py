"""gloo on GPU tensors for multi-rank rehearsals on ONE MI355X.

RCCL refuses two ranks on one device, so the 8-rank layout rehearsals
(scripts/rehearse_layouts_1gpu.sh, ``bench.py --backend gloo``) and the multi-rank
GPU tests run gloo.  gloo has no device path for point-to-point and all-to-all,
so these are staged through host memory here.  Point-to-point stays asynchronous
(a posted receive completes at ``wait()``); all-to-all is blocking.  Debug/rehearsal
only; production runs use RCCL.
"""
from __future__ import annotations

_INSTALLED = [False]


def stage_gloo_cuda_p2p() -> None:
    """Let gloo groups carry CUDA tensors through point-to-point and all-to-all
    by staging them through host memory (idempotent)."""
    if _INSTALLED[0]:
        return
    _INSTALLED[0] = True
    import torch
    import torch.distributed as dist

    real_batch, real_a2a = dist.batch_isend_irecv, dist.all_to_all_single

    class _Done:
        def wait(self):
            return True

        def is_completed(self):
            return True

    class _Staged:
        """The gloo works of one staged batch; ``wait()`` (once) joins them and copies
        every received host buffer into its device tensor."""

        def __init__(self, works, back, keep):
            self.works, self.back, self.keep = works, back, keep

        def wait(self):
            for w in self.works:  # a gloo work must not be waited twice (it can hang)
                w.wait()
            for dst, t in self.back:
                dst.copy_(t)
            self.works, self.back, self.keep = [], [], []
            return True

        def is_completed(self):
            return not self.works

    def batch_isend_irecv(ops):
        # asynchronous like RCCL: receives posted ahead (pipeline mailboxes) must not block
        # the host until their data is used
        if not any(op.tensor.is_cuda for op in ops):
            return real_batch(ops)
        host, back = [], []
        for op in ops:
            t = op.tensor.detach().to("cpu", copy=True)
            host.append(dist.P2POp(op.op, t, op.peer, op.group, op.tag))
            if op.op in (dist.irecv, dist.recv):
                back.append((op.tensor, t))
        return [_Staged(real_batch(host), back, host)]

    def all_to_all_single(output, input, output_split_sizes=None, input_split_sizes=None, group=None,
                          async_op=False):
        if not input.is_cuda:
            return real_a2a(output, input, output_split_sizes, input_split_sizes, group=group, async_op=async_op)
        out_h = torch.empty(output.shape, dtype=output.dtype)
        real_a2a(out_h, input.cpu(), output_split_sizes, input_split_sizes, group=group)
        output.copy_(out_h)
        return _Done() if async_op else None

    dist.batch_isend_irecv = batch_isend_irecv
    dist.all_to_all_single = all_to_all_single
