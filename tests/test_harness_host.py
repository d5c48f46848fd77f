"""CPU: the training harness -- prototxt parsing with the reference's
schema, the CIFAR ResNet + ReplaceModuleTool state_dict layout against the reference's own
(golden from tests/golden/make_golden_harness.py), the torchvision-free CIFAR-10 reader and
loader, the optimizer / LR-schedule construction, and the checkpoint format."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from cim_quantization_amd.harness import config, data, models, train
from cim_quantization_amd.harness.replace import ReplaceModuleTool

EXAMPLE = """
main_file: "examples/classifier_cifar10/main_lsq.py"
arch: "resnet20"
model_source: Local
log_name: "temp"
debug: false
data: "./CIFAR-10"
lr: 0.01
epochs: 100
batch_size: 256
workers: 8
print_freq: 40
evaluate: false
pretrained: true
seed: 0
gpu_id: ANY
nbits_w: 3
nbits_a: 3
nbits_alpha: 8
wbitslice: 1
abitslice: 1
xbar: 128
adcbits: 1.5
stochastic_quant: False
resume : '/nonexistent/resnet20_Conv2dLSQCiMbest.pth.tar'
lr_scheduler: CosineAnnealingLR
optimizer: SGD
sgd {
  weight_decay: 1e-4
  momentum: 0.9
}
"""


def test_prototxt_fields_enums_defaults():
    hp = config.parse_hyperparam(EXAMPLE)
    e = config.eppb
    assert hp.arch == "resnet20" and hp.data == "./CIFAR-10" and hp.epochs == 100 and hp.batch_size == 256
    assert hp.model_source == e.HyperParam.ModelSource.Local and hp.gpu_id == e.GPU.ANY
    assert hp.lr_scheduler == e.LRScheduleType.CosineAnnealingLR and hp.optimizer == e.OptimizerType.SGD
    assert abs(hp.adcbits - 1.5) < 1e-7 and hp.xbar == 128 and hp.nbits_w == 3 and not hp.stochastic_quant
    assert hp.HasField("seed") and hp.seed == 0 and hp.HasField("resume") and not hp.HasField("weight")
    assert abs(hp.sgd.momentum - 0.9) < 1e-7
    assert not hp.HasField("multi_gpu") and hp.multi_gpu.dist_url == "tcp://127.0.0.1:23456"  # defaults
    assert hp.multi_gpu.world_size == -1 and hp.multi_gpu.dist_backend == "nccl"
    assert not hp.HasField("warmup") and hp.warmup.epochs == 10 and hp.step_lr.step_size == 20
    hp2 = config.parse_hyperparam('data: "d"\nlr_scheduler: MultiStepLR\nmulti_step_lr { milestones: 30 milestones: 60 '
                                  'gamma: 0.2 }\nwarmup { epochs: 2 multiplier: 1 }\ncyclic_lr { mode: exp_range }')
    assert list(hp2.multi_step_lr.milestones) == [30, 60] and hp2.HasField("warmup")
    assert hp2.cyclic_lr.mode == e.CyclicLRParam.Mode.exp_range and hp2.lr == pytest.approx(0.1)
    with pytest.raises(Exception):
        config.parse_hyperparam('data: "d"\nno_such_field: 1')
    assert not config.parse_hyperparam("arch: 'x'").IsInitialized()  # required ``data`` missing


def test_resnet20_cim_state_dict_matches_reference():
    from cim_quantization_amd._modules.lsq import Conv2dLSQCiM
    with open(os.path.join(GOLDEN, "harness_resnet20_cim_state.json")) as f:
        ref = json.load(f)
    model = models.resnet20()
    tool = ReplaceModuleTool(model, {"Conv2d": [Conv2dLSQCiM]}, True, **ref["kwargs"])
    tool.replace()
    mine = [[k, list(v.shape), str(v.dtype)] for k, v in model.state_dict().items()]
    assert mine == ref["state"]
    assert [[c.nbits_w, c.nbits_a] for c in tool.convs] == ref["conv_bits"]  # first layer forced to w8a8


def test_replace_keeps_first_layer_float_when_asked():
    from cim_quantization_amd._modules.lsq import Conv2dLSQCiM
    model = models.resnet20()
    w0 = model.layer1[0].conv1.weight.detach().clone()
    ReplaceModuleTool(model, {"Conv2d": [Conv2dLSQCiM]}, False, nbits_w=3, nbits_a=3, xbar=128, adcbits=1.5).replace()
    assert type(model.conv1) is torch.nn.Conv2d
    assert isinstance(model.layer1[0].conv1, Conv2dLSQCiM)
    assert torch.equal(model.layer1[0].conv1.weight.detach(), w0)  # float weights copied


def test_resnet_depths():
    for fn, convs in ((models.resnet20, 19), (models.resnet32, 31), (models.resnet56, 55)):
        m = fn()
        assert sum(isinstance(x, torch.nn.Conv2d) for x in m.modules()) == convs
    assert sum(p.numel() for p in models.resnet20().parameters()) == 269722  # the paper's 0.27M


def test_cifar_binary_reader_and_loader(tmp_path):
    rng = np.random.default_rng(0)
    d = tmp_path / "cifar-10-batches-bin"
    d.mkdir()
    xs, ys = [], []
    for i in range(1, 3):
        x = rng.integers(0, 256, (7, 3, 32, 32), dtype=np.uint8)
        y = rng.integers(0, 10, 7)
        data.write_cifar10_bin(str(d / f"data_batch_{i}.bin"), x, y)
        xs.append(x)
        ys.append(y)
    data.write_cifar10_bin(str(d / "test_batch.bin"), xs[0][:5], ys[0][:5])
    xtr, ytr, xte, yte = data.load_cifar10(str(tmp_path))
    assert np.array_equal(xtr, np.concatenate(xs)) and np.array_equal(ytr, np.concatenate(ys))
    assert xte.shape == (5, 3, 32, 32)
    # DistributedSampler semantics: two ranks cover every sample, equal shares
    seen = []
    for r in range(2):
        ld = data.CifarLoader(xtr, np.arange(14), 4, torch.device("cpu"), train=True, seed=3, rank=r, world=2)
        ld.set_epoch(1)
        seen += torch.cat([yb for _, yb in ld]).tolist()
    assert sorted(seen) == list(range(14))
    val = data.CifarLoader(xte, yte, 2, torch.device("cpu"), train=False)
    xb, _ = next(iter(val))
    mean = torch.tensor(data.MEAN).view(1, 3, 1, 1)
    std = torch.tensor(data.STD).view(1, 3, 1, 1)
    assert torch.allclose(xb, (torch.from_numpy(xte[:2]).float() / 255 - mean) / std)


def test_optimizer_groups_and_schedules():
    from cim_quantization_amd._modules.lsq import Conv2dLSQCiM
    model = models.resnet20()
    ReplaceModuleTool(model, {"Conv2d": [Conv2dLSQCiM]}, True, nbits_w=3, nbits_a=3, xbar=128, adcbits=1.5).replace()
    hp = config.parse_hyperparam(EXAMPLE)
    opt = train.get_optimizer(model, hp)
    names = {id(p): n for n, p in model.named_parameters()}
    assert all("alpha" in names[id(p)] for p in opt.param_groups[0]["params"])  # no weight decay on step sizes
    assert opt.param_groups[0]["weight_decay"] == 0.0 and opt.param_groups[1]["weight_decay"] == pytest.approx(1e-4)
    sch = train.get_lr_scheduler(opt, hp)
    lrs = []
    for _ in range(3):
        lrs.append(opt.param_groups[1]["lr"])
        sch.step()
    assert lrs[0] == pytest.approx(0.01) and lrs[2] == pytest.approx(0.01 * (1 + np.cos(np.pi * 2 / 100)) / 2, rel=1e-5)
    hp.warmup.epochs, hp.warmup.multiplier = 4, 10.0
    opt = train.get_optimizer(model, hp)
    sch = train.get_lr_scheduler(opt, hp)
    lrs = []
    for _ in range(4):
        lrs.append(opt.param_groups[1]["lr"])
        sch.step()
    assert lrs == pytest.approx([0.01 * ((10 - 1) * e / 4 + 1) for e in range(4)], rel=1e-5)


def test_checkpoint_round_trip(tmp_path):
    model = models.resnet20()
    opt = torch.optim.SGD(model.parameters(), 0.1, momentum=0.9)
    model(torch.randn(2, 3, 32, 32)).sum().backward()
    opt.step()
    prefix = str(tmp_path / "resnet20_Conv2dLSQCiM")
    train.save_checkpoint({"epoch": 1, "arch": "resnet20_Conv2dLSQCiM", "state_dict": model.state_dict(),
                           "best_acc1": 12.5, "optimizer": opt.state_dict()}, True, prefix)
    ck = torch.load(prefix + "best.pth.tar", map_location="cpu", weights_only=True)
    assert ck["epoch"] == 1 and ck["best_acc1"] == 12.5
    m2 = models.resnet20()
    m2.load_state_dict(ck["state_dict"])
    assert all(torch.equal(a, b) for a, b in zip(model.state_dict().values(), m2.state_dict().values()))


def test_resume_accepts_reference_ddp_keys():
    """main_lsq.py:121 saves the DDP-wrapped model ('module.' keys); resume strips or adds the
    prefix to match, and a checkpoint with no matching key is an error, not a silent no-op."""
    src = models.resnet20()
    ddp_state = {"module." + k: v for k, v in src.state_dict().items()}
    dst = models.resnet20()
    train.load_resume_state(dst, ddp_state)
    assert all(torch.equal(a, b) for a, b in zip(src.state_dict().values(), dst.state_dict().values()))

    class Wrap(torch.nn.Module):
        def __init__(self, m):
            super().__init__()
            self.module = m
    wrapped = Wrap(models.resnet20())
    train.load_resume_state(wrapped, src.state_dict())
    assert all(torch.equal(a, b) for a, b in zip(src.state_dict().values(), wrapped.module.state_dict().values()))
    with pytest.raises(RuntimeError, match="no checkpoint key"):
        train.load_resume_state(models.resnet20(), {"foo.bar": torch.zeros(1)})
