"""GPU: the prototxt-driven CIFAR-10 launcher (cim_quantization_amd.harness.train, the flow of
examples/classifier_cifar10/main_lsq.py) end to end on synthetic CIFAR-10 binary batches:
ResNet-20 with every conv replaced by Conv2dLSQCiM (first layer w8a8), a few SGD steps, a
checkpoint in the reference's format, and an evaluate-only run resumed from it."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

PROTO = """
arch: "resnet20"
model_source: Local
log_name: "{log}"
data: "{data}"
lr: 0.05
epochs: 2
batch_size: 64
print_freq: 1
seed: 0
gpu_id: ANY
nbits_w: 3
nbits_a: 3
nbits_alpha: 8
wbitslice: 1
abitslice: 1
xbar: 128
adcbits: 1.5
lr_scheduler: CosineAnnealingLR
optimizer: SGD
sgd {{ weight_decay: 1e-4 momentum: 0.9 }}
{extra}
"""


def _data(root):
    from cim_quantization_amd.harness.data import write_cifar10_bin
    d = os.path.join(root, "cifar-10-batches-bin")
    os.makedirs(d)
    rng = np.random.default_rng(0)
    y = rng.integers(0, 10, 256)
    # class-dependent mean colour so a few steps can fit something
    x = np.clip(rng.normal(100 + 12 * y[:, None, None, None], 40, (256, 3, 32, 32)), 0, 255).astype(np.uint8)
    write_cifar10_bin(os.path.join(d, "data_batch_1.bin"), x, y)
    write_cifar10_bin(os.path.join(d, "test_batch.bin"), x[:128], y[:128])


def test_train_checkpoint_resume(cuda_device, tmp_path, capsys):
    from cim_quantization_amd.harness import train
    from cim_quantization_amd._modules.lsq import Conv2dLSQCiM
    _data(str(tmp_path))
    log = str(tmp_path / "run")
    hp1 = tmp_path / "train.prototxt"
    hp1.write_text(PROTO.format(log=log, data=str(tmp_path), extra=""))
    best = train.main(["--hp", str(hp1), "--max-steps", "3", "--max-val-steps", "2"])
    out = capsys.readouterr().out
    assert "epoch 1:" in out and np.isfinite(best)
    losses = [float(l.split("loss ")[1].split()[0]) for l in out.splitlines() if l.startswith("Epoch [")]
    assert len(losses) == 6 and all(np.isfinite(losses))
    ck_path = os.path.join(log, "resnet20_Conv2dLSQCiMcheckpoint.pth.tar")
    ck = torch.load(ck_path, map_location="cpu", weights_only=True)
    assert ck["epoch"] == 2 and ck["arch"] == "resnet20_Conv2dLSQCiM" and "optimizer" in ck
    sd = ck["state_dict"]
    assert sd["conv1.alpha_cim"].shape == (1, 1, 8, 8, 1, 16) and float(sd["conv1.init_state"]) == 1.0
    assert all(torch.isfinite(v).all() for v in sd.values() if v.is_floating_point())
    # evaluate-only run resumed from the checkpoint: same weights, same accuracy as the last validation
    hp2 = tmp_path / "eval.prototxt"
    hp2.write_text(PROTO.format(log=log, data=str(tmp_path), extra=f'evaluate: true\nresume: "{ck_path}"'))
    acc = train.main(["--hp", str(hp2), "--max-val-steps", "2"])
    model, _ = train.build_model(train.load_hyperparam(str(hp2)), cuda_device)
    assert isinstance(model.layer3[2].conv2, Conv2dLSQCiM)
    assert torch.equal(model.layer3[2].conv2.alpha_cim.detach().cpu(), sd["layer3.2.conv2.alpha_cim"])
    assert np.isfinite(acc)
