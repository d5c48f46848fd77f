"""The reference's prototxt hyper-parameter format (proto/efficient_pytorch.proto, package
``efficient_pytorch``), read with google.protobuf's own text-format parser.

There is no protoc in this image, so the schema is declared here field by field (names,
numbers, labels, types, defaults and enums as the .proto defines them) and turned into real
protobuf message classes at import time through a FileDescriptorProto: ``hp.HasField('seed')``,
``hp.multi_gpu.dist_url`` defaults, ``eppb.GPU.ANY``, ``eppb.HyperParam.ModelSource.Local`` and
``text_format.Merge`` behave as with the reference's generated efficient_pytorch_pb2
(examples/__init__.py:107-114 reads configs that way).

    from cim_quantization_amd.harness.config import eppb, load_hyperparam
    hp = load_hyperparam("resnet_w3a3.prototxt")
"""
from __future__ import annotations

import types

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory, text_format

_FD = descriptor_pb2.FieldDescriptorProto
_T = dict(string=_FD.TYPE_STRING, bool=_FD.TYPE_BOOL, float=_FD.TYPE_FLOAT, int32=_FD.TYPE_INT32,
          enum=_FD.TYPE_ENUM, message=_FD.TYPE_MESSAGE)
_L = dict(optional=_FD.LABEL_OPTIONAL, required=_FD.LABEL_REQUIRED, repeated=_FD.LABEL_REPEATED)

PACKAGE = "efficient_pytorch"

# top-level enums: name -> [(value name, number)]
ENUMS = {
    "GPU": [("ANY", 1), ("NONE", 2)],
    "Qmode": [("layer_wise", 1), ("kernel_wise", 2)],
    "CimMode": [("column_wise", 1), ("bit_wise", 2)],
    "OptimizerType": [("SGD", 1), ("Adam", 2)],
    "LRScheduleType": [("StepLR", 1), ("MultiStepLR", 2), ("CosineAnnealingLR", 3), ("CyclicLR", 4)],
}

# messages: name -> (fields, nested enums); field = (label, type, name, number, type_name, default)
MESSAGES = {
    "HyperParam": ([
        ("optional", "string", "main_file", 1, None, "examples/classifier_imagenet/main.py"),
        ("optional", "string", "arch", 2, None, "alexnet"),
        ("optional", "enum", "model_source", 3, ".efficient_pytorch.HyperParam.ModelSource", None),
        ("optional", "string", "log_name", 4, None, "template"),
        ("required", "string", "data", 5, None, None),
        ("optional", "bool", "debug", 6, None, None),
        ("optional", "bool", "overfit_test", 7, None, None),
        ("optional", "float", "lr", 10, None, "0.1"),
        ("optional", "int32", "epochs", 11, None, "90"),
        ("optional", "int32", "batch_size", 12, None, "256"),
        ("optional", "int32", "workers", 13, None, "4"),
        ("optional", "int32", "print_freq", 14, None, "50"),
        ("optional", "int32", "log_freq", 322, None, "40"),
        ("optional", "bool", "evaluate", 15, None, None),
        ("optional", "bool", "pretrained", 16, None, None),
        ("optional", "string", "pretrained_location", 321, None, None),
        ("optional", "int32", "seed", 17, None, None),
        ("optional", "bool", "export_onnx", 18, None, None),
        ("optional", "string", "resume", 19, None, None),
        ("optional", "string", "weight", 22, None, None),
        ("optional", "enum", "gpu_id", 20, ".efficient_pytorch.GPU", None),
        ("optional", "message", "multi_gpu", 21, ".efficient_pytorch.MultiGPU", None),
        ("optional", "enum", "qmode", 50, ".efficient_pytorch.Qmode", None),
        ("optional", "int32", "nbits_w", 51, None, "4"),
        ("optional", "int32", "nbits_a", 52, None, "4"),
        ("optional", "int32", "nbits_alpha", 520, None, "8"),
        ("optional", "int32", "wbitslice", 53, None, "1"),
        ("optional", "int32", "abitslice", 54, None, "1"),
        ("optional", "int32", "xbar", 55, None, "64"),
        ("optional", "float", "adcbits", 56, None, "6"),
        ("optional", "bool", "signed_xbar", 58, None, None),
        ("optional", "bool", "stochastic_quant", 59, None, None),
        ("optional", "enum", "cimmode", 57, ".efficient_pytorch.CimMode", None),
        ("optional", "message", "warmup", 99, ".efficient_pytorch.Warmup", None),
        ("optional", "enum", "lr_scheduler", 100, ".efficient_pytorch.LRScheduleType", None),
        ("optional", "message", "step_lr", 101, ".efficient_pytorch.StepLRParam", None),
        ("optional", "message", "multi_step_lr", 102, ".efficient_pytorch.MultiStepLRParam", None),
        ("optional", "message", "cyclic_lr", 103, ".efficient_pytorch.CyclicLRParam", None),
        ("optional", "enum", "optimizer", 200, ".efficient_pytorch.OptimizerType", None),
        ("optional", "message", "sgd", 201, ".efficient_pytorch.SGDParam", None),
        ("optional", "message", "adam", 202, ".efficient_pytorch.AdamParam", None),
    ], {"ModelSource": [("TorchVision", 1), ("PyTorchCV", 2), ("Local", 3)]}),
    "MultiGPU": ([
        ("optional", "int32", "world_size", 1, None, "-1"),
        ("optional", "int32", "rank", 2, None, "0"),
        ("optional", "string", "dist_url", 3, None, "tcp://127.0.0.1:23456"),
        ("optional", "string", "dist_backend", 4, None, "nccl"),
        ("optional", "bool", "multiprocessing_distributed", 5, None, None),
    ], {}),
    "SGDParam": ([
        ("optional", "float", "weight_decay", 1, None, "1e-4"),
        ("optional", "float", "momentum", 2, None, "0.9"),
    ], {}),
    "AdamParam": ([("optional", "float", "weight_decay", 1, None, "1e-4")], {}),
    "Warmup": ([
        ("optional", "int32", "epochs", 1, None, "10"),
        ("optional", "float", "multiplier", 2, None, "10"),
    ], {}),
    "StepLRParam": ([
        ("optional", "int32", "step_size", 3, None, "20"),
        ("optional", "float", "gamma", 4, None, "0.1"),
    ], {}),
    "MultiStepLRParam": ([
        ("repeated", "int32", "milestones", 3, None, None),
        ("optional", "float", "gamma", 4, None, "0.1"),
    ], {}),
    "CyclicLRParam": ([
        ("optional", "float", "base_lr", 1, None, None),
        ("optional", "float", "max_lr", 2, None, None),
        ("optional", "int32", "step_size_up", 3, None, "2000"),
        ("optional", "int32", "step_size_down", 4, None, None),
        ("optional", "enum", "mode", 5, ".efficient_pytorch.CyclicLRParam.Mode", None),
        ("optional", "float", "gamma", 6, None, "1.0"),
    ], {"Mode": [("triangular", 1), ("triangular2", 2), ("exp_range", 3)]}),
}


def _enum(proto, name, values):
    e = proto.add()
    e.name = name
    for vn, num in values:
        v = e.value.add()
        v.name, v.number = vn, num


def _file_descriptor():
    fd = descriptor_pb2.FileDescriptorProto()
    fd.name = "cim_quantization_amd/efficient_pytorch.proto"
    fd.package = PACKAGE
    fd.syntax = "proto2"
    for name, values in ENUMS.items():
        _enum(fd.enum_type, name, values)
    for name, (fields, nested) in MESSAGES.items():
        m = fd.message_type.add()
        m.name = name
        for en, values in nested.items():
            _enum(m.enum_type, en, values)
        for label, typ, fname, num, type_name, default in fields:
            f = m.field.add()
            f.name, f.number = fname, num
            f.label, f.type = _L[label], _T[typ]
            if type_name:
                f.type_name = type_name
            if default is not None:
                f.default_value = default
    return fd


_POOL = descriptor_pool.DescriptorPool()
_FILE = _POOL.Add(_file_descriptor())


def _build_module():
    mod = types.ModuleType("efficient_pytorch_pb2")
    for name in MESSAGES:
        setattr(mod, name, message_factory.GetMessageClass(_POOL.FindMessageTypeByName(f"{PACKAGE}.{name}")))
    for name in ENUMS:
        ed = _POOL.FindEnumTypeByName(f"{PACKAGE}.{name}")
        setattr(mod, name, types.SimpleNamespace(**{v.name: v.number for v in ed.values}, Name=ed.values_by_number))
        for v in ed.values:  # top-level enum values are module attributes in generated code
            setattr(mod, v.name, v.number)
    return mod


eppb = _build_module()


def load_hyperparam(path: str):
    """Parse a prototxt into a HyperParam (text_format.Merge, as get_hyperparam does)."""
    hp = eppb.HyperParam()
    with open(path) as f:
        text_format.Merge(f.read(), hp)
    return hp


def parse_hyperparam(text: str):
    hp = eppb.HyperParam()
    text_format.Merge(text, hp)
    return hp
