"""HIP-graph capture of the operator (the MI355X answer to a tracing compiler for launch-bound
loops): forward + backward through `flash_attn_func` captured with torch.cuda.graph and replayed
give the same bits as eager calls -- every kernel is deterministic and launches on the current
stream with no host synchronisation or host-side allocation outside torch's graph pool.
"""
import pytest
import torch

from tests.core import generate_attention_mask, generate_test_data


def _step(q, k, v, do, causal, mask=None):
    from fa2_triton_amd import flash_attn_func

    out = flash_attn_func(q, k, v, attention_mask=mask, causal=causal)
    dq, dk, dv = torch.autograd.grad(out, (q, k, v), do)
    return out, dq, dk, dv


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("shape", [(2, 8, 8, 512, 128), (1, 16, 1, 700, 128), (2, 4, 2, 333, 64)],
                         ids=["mha-d128", "mqa-split-d128", "gqa-d64"])
@pytest.mark.parametrize("use_mask", [False, True])
def test_graph_replay_matches_eager(causal, shape, use_mask):
    b, hq, hkv, s, d = shape
    q, k, v, do = generate_test_data(b, hq, hkv, s, s, d, torch.bfloat16)
    mask = generate_attention_mask(q) if use_mask else None
    eager = _step(q, k, v, do, causal, mask)
    # the captured step gets leaves of its own: an AccumulateGrad node created on the default
    # stream (by the eager call above) must not be reused inside the capture
    q, k, v = (t.detach().clone().requires_grad_() for t in (q, k, v))

    # static inputs, warmed up on a side stream as torch.cuda.graph requires
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            _step(q, k, v, do, causal, mask)
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        captured = _step(q, k, v, do, causal, mask)
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    for name, x, y in zip(("out", "dq", "dk", "dv"), captured, eager):
        assert torch.equal(x, y), name

    # new inputs copied into the static tensors: the replay follows them
    q2, k2, v2, do2 = generate_test_data(b, hq, hkv, s, s, d, torch.bfloat16, seed=7)
    with torch.no_grad():
        q.copy_(q2)
        k.copy_(k2)
        v.copy_(v2)
        do.copy_(do2)
    graph.replay()
    torch.cuda.synchronize()
    fresh = _step(*(t.detach().clone().requires_grad_() for t in (q, k, v)), do, causal, mask)
    for name, x, y in zip(("out", "dq", "dk", "dv"), captured, fresh):
        assert torch.equal(x, y), name
