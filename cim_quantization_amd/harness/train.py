"""CIFAR-10 training launcher driven by the reference's prototxt (examples/classifier_cifar10/
main_lsq.py and the helpers of examples/__init__.py), on MI355X with Conv2dLSQCiM layers.

    python -m cim_quantization_amd.harness.train --hp resnet_w3a3.prototxt
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m cim_quantization_amd.harness.train --hp ...

Flow as main_lsq.py: seed (main_s1_set_seed), float ResNet from models.py, optional ``weight``
load, ReplaceModuleTool({'Conv2d': [Conv2dLSQCiM]}, replace_first_layer=True, the CiM kwargs of
the prototxt), optional ``resume`` (state_dict, strict=False), DistributedDataParallel when
launched with WORLD_SIZE > 1 (one process per GPU, RCCL; the per-process batch is batch_size /
world as distributed_model does), SGD with the alpha/scale parameters excluded from weight
decay (add_weight_decay) or Adam, the prototxt's LR schedule (+ gradual warmup), validate before
training and after every epoch, and checkpoints in the reference's format
({'epoch', 'arch', 'state_dict', 'best_acc1', 'optimizer'}, <log_name>/<arch>checkpoint.pth.tar
and ...best.pth.tar).  Checkpoints are read back with torch.load(weights_only=True).
Out of scope: tensorboard logging, ONNX export, ptflops, BN fusion,
ImageNet / MNIST loaders, the script-copying bookkeeping of main_lsq.py.
"""
from __future__ import annotations

import argparse
import os
import random
import shutil
import time

import torch
import torch.distributed as dist
import torch.nn as nn

from . import models
from .config import eppb, load_hyperparam
from .data import CifarLoader, load_cifar10
from .replace import ReplaceModuleTool

WEIGHT_DECAY_SKIP = ("expand_", "running_scale", "alpha", "standard_threshold", "nbits")  # get_optimizer


def get_base_parser():
    p = argparse.ArgumentParser(description="CiM-quantised CIFAR-10 training on MI355X")
    p.add_argument("--hp", type=str, required=True, help="prototxt hyper-parameter file")
    p.add_argument("--start-epoch", default=0, type=int)
    p.add_argument("--max-steps", default=0, type=int, help="stop each epoch after this many steps (0: all)")
    p.add_argument("--max-val-steps", default=0, type=int)
    return p


def set_seed(hp):
    if hp.HasField("seed"):
        random.seed(hp.seed)
        torch.manual_seed(hp.seed)


def add_weight_decay(model, weight_decay, skip_keys=WEIGHT_DECAY_SKIP):
    decay, no_decay = [], []
    for name, p in model.named_parameters():
        if not p.requires_grad:
            continue
        (no_decay if any(k in name for k in skip_keys) else decay).append(p)
    return [{"params": no_decay, "weight_decay": 0.0}, {"params": decay, "weight_decay": weight_decay}]


def get_optimizer(model, hp):
    if hp.optimizer == eppb.OptimizerType.SGD:
        return torch.optim.SGD(add_weight_decay(model, hp.sgd.weight_decay), hp.lr, momentum=hp.sgd.momentum)
    if hp.optimizer == eppb.OptimizerType.Adam:
        return torch.optim.Adam(model.parameters(), lr=hp.lr, weight_decay=hp.adam.weight_decay)
    raise NotImplementedError(f"optimizer {hp.optimizer}")


class GradualWarmup(torch.optim.lr_scheduler.LRScheduler):
    """Linear warm-up to base_lr * multiplier over ``total_epoch`` epochs, then ``after`` on the
    raised base (the GradualWarmupScheduler the reference imports from warmup_scheduler)."""

    def __init__(self, optimizer, multiplier, total_epoch, after):
        self.multiplier, self.total_epoch, self.after = multiplier, total_epoch, after
        self.finished = False
        super().__init__(optimizer)

    def get_lr(self):
        if self.last_epoch > self.total_epoch:
            if not self.finished:
                self.after.base_lrs = [b * self.multiplier for b in self.base_lrs]
                self.finished = True
            return self.after.get_last_lr()
        if self.multiplier == 1.0:
            return [b * float(self.last_epoch) / self.total_epoch for b in self.base_lrs]
        return [b * ((self.multiplier - 1.0) * self.last_epoch / self.total_epoch + 1.0) for b in self.base_lrs]

    def step(self, epoch=None):
        if self.finished and self.after is not None:
            self.after.step()
            self._last_lr = self.after.get_last_lr()
            self.last_epoch += 1
        else:
            super().step()


def get_lr_scheduler(optimizer, hp):
    t = hp.lr_scheduler
    if t == eppb.LRScheduleType.CosineAnnealingLR:
        nxt = torch.optim.lr_scheduler.CosineAnnealingLR(optimizer, T_max=hp.epochs)
    elif t == eppb.LRScheduleType.StepLR:
        nxt = torch.optim.lr_scheduler.StepLR(optimizer, step_size=hp.step_lr.step_size, gamma=hp.step_lr.gamma)
    elif t == eppb.LRScheduleType.MultiStepLR:
        nxt = torch.optim.lr_scheduler.MultiStepLR(optimizer, milestones=list(hp.multi_step_lr.milestones),
                                                   gamma=hp.multi_step_lr.gamma)
    elif t == eppb.LRScheduleType.CyclicLR:
        c = hp.cyclic_lr
        mode = {eppb.CyclicLRParam.Mode.triangular: "triangular", eppb.CyclicLRParam.Mode.triangular2: "triangular2",
                eppb.CyclicLRParam.Mode.exp_range: "exp_range"}[c.mode]
        nxt = torch.optim.lr_scheduler.CyclicLR(optimizer, base_lr=c.base_lr, max_lr=c.max_lr,
                                                step_size_up=c.step_size_up,
                                                step_size_down=c.step_size_down if c.HasField("step_size_down") else None,
                                                mode=mode, gamma=c.gamma)
    else:
        raise NotImplementedError(f"lr_scheduler {t}")
    if not hp.HasField("warmup"):
        return nxt
    return GradualWarmup(optimizer, hp.warmup.multiplier, hp.warmup.epochs, nxt)


def build_model(hp, device):
    """Float ResNet -> weight file -> CiM replacement -> resume, as process_model."""
    from .._modules.lsq import Conv2dLSQCiM
    if hp.model_source != eppb.HyperParam.ModelSource.Local:
        raise NotImplementedError("model_source must be Local (torchvision / pytorchcv are not available)")
    model = models.__dict__[hp.arch](pretrained=hp.pretrained, pretrained_location=hp.pretrained_location or None)
    if hp.HasField("weight") and os.path.isfile(hp.weight):
        model.load_state_dict(torch.load(hp.weight, map_location="cpu", weights_only=True))
    tool = ReplaceModuleTool(model, {"Conv2d": [Conv2dLSQCiM]}, True, nbits_w=hp.nbits_w, nbits_a=hp.nbits_a,
                             nbits_alpha=hp.nbits_alpha, wbitslice=hp.wbitslice, abitslice=hp.abitslice, xbar=hp.xbar,
                             adcbits=hp.adcbits, signed_xbar=hp.signed_xbar, stochastic_quant=hp.stochastic_quant)
    tool.replace()
    arch = f"{hp.arch}_Conv2dLSQCiM"
    if hp.HasField("resume") and os.path.isfile(hp.resume):
        ck = torch.load(hp.resume, map_location="cpu", weights_only=True)
        load_resume_state(model, ck.get("state_dict", ck))
    return model.to(device), arch


def load_resume_state(model, state):
    """Resume from a checkpoint written here (the bare model's keys) or by the reference's
    main_lsq.py under DDP (main_lsq.py:121 saves the wrapped model, keys prefixed 'module.').
    The prefix is stripped or added to match ``model``; non-strict like the reference's resume,
    but a checkpoint none of whose keys match is an error rather than a silent no-op."""
    own = model.state_dict().keys()
    wrapped = any(k.startswith("module.") for k in own)
    fixed = {}
    for k, v in state.items():
        bare = k[len("module."):] if k.startswith("module.") else k
        fixed[("module." + bare) if wrapped else bare] = v
    res = model.load_state_dict(fixed, strict=False)
    if fixed and len(res.unexpected_keys) == len(fixed):
        raise RuntimeError("resume: no checkpoint key matches the model (%d keys, e.g. %r)"
                           % (len(fixed), next(iter(fixed))))
    return res


def accuracy(output, target, topk=(1,)):
    with torch.no_grad():
        maxk = max(topk)
        _, pred = output.topk(maxk, 1, True, True)
        correct = pred.t().eq(target.view(1, -1).expand_as(pred.t()))
        return [correct[:k].reshape(-1).float().sum().mul_(100.0 / target.size(0)) for k in topk]


def train_epoch(loader, model, criterion, optimizer, epoch, hp, max_steps=0, log=print):
    model.train()
    t0 = time.time()
    seen, loss_sum, top1 = 0, 0.0, 0.0
    for i, (x, y) in enumerate(loader):
        out = model(x)
        loss = criterion(out, y)
        a1, = accuracy(out, y, (1,))
        optimizer.zero_grad()
        loss.backward()
        optimizer.step()
        n = y.numel()
        seen += n
        loss_sum += loss.item() * n
        top1 += a1.item() * n
        if i % max(hp.print_freq, 1) == 0:
            log(f"Epoch [{epoch}] {i}/{len(loader)} loss {loss.item():.4f} acc1 {a1.item():.2f} "
                f"lr {optimizer.param_groups[0]['lr']:.5f} {time.time() - t0:.1f}s")
        if hp.overfit_test or (max_steps and i + 1 >= max_steps):
            break
    return loss_sum / max(seen, 1), top1 / max(seen, 1)


def validate(loader, model, criterion, hp, max_steps=0):
    model.eval()
    seen, loss_sum, c1, c5 = 0, 0.0, 0.0, 0.0
    with torch.no_grad():
        for i, (x, y) in enumerate(loader):
            out = model(x)
            a1, a5 = accuracy(out, y, (1, 5))
            n = y.numel()
            seen += n
            loss_sum += criterion(out, y).item() * n
            c1 += a1.item() * n
            c5 += a5.item() * n
            if hp.overfit_test or (max_steps and i + 1 >= max_steps):
                break
    return c1 / max(seen, 1), c5 / max(seen, 1), loss_sum / max(seen, 1)


def save_checkpoint(state, is_best, prefix, filename="checkpoint.pth.tar"):
    torch.save(state, prefix + filename)
    if is_best:
        shutil.copyfile(prefix + filename, prefix + "best.pth.tar")


def main(argv=None):
    args = get_base_parser().parse_args(argv)
    hp = load_hyperparam(args.hp)
    set_seed(hp)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    if hp.gpu_id == eppb.GPU.NONE:
        raise RuntimeError("gpu_id NONE: the CiM layers run on ROCm devices only")
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    if distributed:
        backend = hp.multi_gpu.dist_backend if hp.HasField("multi_gpu") else "nccl"
        dist.init_process_group(backend=backend, init_method="env://", world_size=world, rank=rank)
    model, arch = build_model(hp, device)
    batch = hp.batch_size // world if distributed else hp.batch_size
    if distributed:
        model = nn.parallel.DistributedDataParallel(model, device_ids=[local])
    criterion = nn.CrossEntropyLoss().to(device)
    optimizer = get_optimizer(model, hp)
    scheduler = get_lr_scheduler(optimizer, hp)
    xtr, ytr, xte, yte = load_cifar10(hp.data)
    seed = hp.seed if hp.HasField("seed") else 0
    train_loader = CifarLoader(xtr, ytr, batch, device, train=True, seed=seed, rank=rank, world=world)
    val_loader = CifarLoader(xte, yte, batch, device, train=False)
    log = print if rank == 0 else (lambda *a, **k: None)
    if hp.evaluate:
        acc1, acc5, _ = validate(val_loader, model, criterion, hp, args.max_val_steps)
        log(f" * Acc@1 {acc1:.3f} Acc@5 {acc5:.3f}")
        return acc1
    for _ in range(args.start_epoch):
        scheduler.step()
    best = 0.0
    if rank == 0:
        os.makedirs(hp.log_name, exist_ok=True)
    acc1, acc5, _ = validate(val_loader, model, criterion, hp, args.max_val_steps)  # main_lsq.py validates first
    log(f"before training: val acc1 {acc1:.3f} acc5 {acc5:.3f}")
    acc1 = 0.0
    for epoch in range(args.start_epoch, hp.epochs):
        train_loader.set_epoch(epoch)
        loss, tacc = train_epoch(train_loader, model, criterion, optimizer, epoch, hp, args.max_steps, log)
        scheduler.step()
        acc1, acc5, vloss = validate(val_loader, model, criterion, hp, args.max_val_steps)
        log(f"epoch {epoch}: train loss {loss:.4f} acc1 {tacc:.2f}  val acc1 {acc1:.3f} acc5 {acc5:.3f}")
        is_best = acc1 > best
        best = max(acc1, best)
        if rank == 0:
            sd = (model.module if distributed else model).state_dict()
            save_checkpoint({"epoch": epoch + 1, "arch": arch, "state_dict": sd, "best_acc1": best,
                             "optimizer": optimizer.state_dict()}, is_best, f"{hp.log_name}/{arch}")
    if distributed:
        dist.destroy_process_group()
    return best


if __name__ == "__main__":
    main()
