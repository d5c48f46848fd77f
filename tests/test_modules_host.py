"""CPU: the drop-in module surface keeps the reference's construction / state contract
(parameter and buffer names, shapes, dtypes, binary_mask, kwargs) and refuses to run
on CPU tensors (no CPU fallback in the product path)."""
import pytest
import torch

import cim_quantization_amd._modules as my_nn
from oracle import cim_module_oracle as cmo

CONFIGS = [
    dict(C=16, O=16, k=3, s=1, p=1, bias=False, nbits_w=3, nbits_a=3, xbar=128, adcbits=1.5),
    dict(C=3, O=16, k=3, s=1, p=1, bias=False, nbits_w=8, nbits_a=8, xbar=128, adcbits=1.5),
    dict(C=32, O=64, k=3, s=2, p=1, bias=False, nbits_w=3, nbits_a=3, xbar=64, adcbits=1),
    dict(C=16, O=16, k=3, s=1, p=1, bias=True, nbits_w=2, nbits_a=2, xbar=64, adcbits=4),
    dict(C=64, O=32, k=1, s=1, p=0, bias=False, nbits_w=4, nbits_a=4, xbar=32, adcbits=1.5),
]


def _make(cls, c):
    return cls(c["C"], c["O"], c["k"], c["s"], c["p"], 1, groups=1, bias=c["bias"], nbits_w=c["nbits_w"],
               nbits_a=c["nbits_a"], nbits_alpha=8, wbitslice=1, abitslice=1, xbar=c["xbar"],
               adcbits=c["adcbits"], signed_xbar=True, stochastic_quant=False)


@pytest.mark.parametrize("c", CONFIGS)
def test_state_dict_contract(c):
    mine = _make(my_nn.Conv2dLSQCiM, c)
    ref = _make(cmo.OracleConv2dLSQCiM, c)
    sm, sr = mine.state_dict(), ref.state_dict()
    assert list(sm.keys()) == list(sr.keys())
    for k in sm:
        assert sm[k].shape == sr[k].shape and sm[k].dtype == sr[k].dtype, k
    assert torch.equal(mine.binary_mask, ref.binary_mask)
    assert mine.binary_mask.dtype == torch.int8
    assert mine.num_xbars == ref.num_xbars
    # checkpoints move between the two
    mine.load_state_dict(sr)


def test_kwargs_defaults_and_names():
    m = my_nn.Conv2dLSQCiM(16, 16, 3, 1, 1, nbits_w=3, nbits_a=3, xbar=128, adcbits=1.5, signed_xbar=False)
    assert m.kwargs_q["mode"] == my_nn.Qmodes.layer_wise
    assert m.kwargs_q["cimmode"] == my_nn.Qmodes_cim.bit_wise
    assert (m.alpha_cim.shape == (1, 2, 3, 3, 1, 16))
    for name in ["Conv2dLSQ", "LinearLSQ", "ActLSQ", "Conv2dLSQCiM", "Qmodes", "_Conv2dQ", "_LinearQ",
                 "_ActQ", "truncation", "get_sparsity_mask", "FunStopGradient", "round_pass", "grad_scale",
                 "Qmodes_cim", "_Conv2dQCiM", "get_cim_output_signed"]:
        assert hasattr(my_nn, name), name


def test_cpu_tensors_are_refused():
    m = _make(my_nn.Conv2dLSQCiM, CONFIGS[0])
    m.train()
    with pytest.raises(RuntimeError, match="ROCm"):
        m(torch.relu(torch.randn(2, 16, 8, 8)))


def test_grad_scale_and_round_pass_values():
    a = torch.tensor([0.123456789], requires_grad=True)
    y = my_nn.grad_scale(a, 0.01)
    y.backward()
    assert abs(a.grad.item() - 0.01) < 1e-9
    v = torch.tensor([0.5, 1.5, 2.5, -0.5, 2.49], requires_grad=True)
    r = my_nn.round_pass(v)
    assert r.tolist() == [0.0, 2.0, 2.0, -0.0, 2.0]
    r.sum().backward()
    assert v.grad.tolist() == [1.0] * 5


def test_plain_modules_host_flag_mirror():
    """Conv2dLSQ / ActLSQ read init_state / signed once (no device sync per forward); any in-place
    write to the buffers (load_state_dict, GradBucket.broadcast_from, torch DDP's per-forward buffer
    broadcast) bumps their version counter and the mirror re-reads them."""
    from cim_quantization_amd._modules.lsq import ActLSQ, Conv2dLSQ
    act, conv = ActLSQ(nbits_a=4), Conv2dLSQ(4, 4, 3, nbits_w=4)
    assert act._flags() == [False, False] and conv._flags() == [False, False]
    sd = act.state_dict()
    sd["init_state"].fill_(1)
    sd["signed"].fill_(1)
    act.load_state_dict(sd)
    assert act._flags() == [True, True]
    assert act._range() == (-8, 7)
    with torch.no_grad():
        conv.init_state.fill_(1)
    assert conv._flags()[0] is True  # a direct in-place write is seen
    with torch.no_grad():
        act.signed.copy_(torch.zeros_like(act.signed))  # what DDP's broadcast from rank 0 does
    assert act._flags() == [True, False] and act._range() == (0, 15)
