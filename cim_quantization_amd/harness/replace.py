"""Module replacement (utils/wrapper/replace_module.py ReplaceModuleTool): swap every
nn.Conv2d / nn.Linear of a float model for the quantised class of ``replace_map``, copying the
float weights.  With ``replace_first_layer`` the first conv is replaced too and built 8-bit
(nbits_w = nbits_a = 8, replace_module.py:83-95); without it the first conv stays float.
A two-entry map value [Act, Conv] inserts Sequential(Act, Conv).
"""
from __future__ import annotations

import torch.nn as nn

__all__ = ["ReplaceModuleTool"]


class ReplaceModuleTool:
    def __init__(self, model, replace_map, replace_first_layer, **kwargs):
        self.model = model
        self.replace_map = replace_map
        self.replace_first_layer = replace_first_layer
        self.kwargs = kwargs
        self.is_first = True
        self.acts, self.convs, self.linears = [], [], []

    def replace(self):
        self._walk(self.model)
        return self.model

    def _walk(self, parent):
        for name, child in list(parent._modules.items()):
            if isinstance(child, (nn.Linear, nn.Conv2d)):
                parent._modules[name] = self._replace(child)
            elif len(child._modules) > 0:
                self._walk(child)

    @staticmethod
    def _split(entry, base):
        if isinstance(entry, (list, tuple)):
            if len(entry) == 2:
                return entry[0], entry[1]
            if len(entry) == 1:
                return None, entry[0]
            raise ValueError("replace_map entries take [Module] or [Act, Module]")
        return None, entry

    def _replace(self, m):
        if isinstance(m, nn.Linear) and "Linear" in self.replace_map:
            act_cls, cls = self._split(self.replace_map["Linear"], nn.Linear)
            q = cls(m.in_features, m.out_features, bias=m.bias is not None, **self.kwargs)
            self.linears.append(q)
            q.weight.data.copy_(m.weight.data)
            if m.bias is not None:
                q.bias.data.copy_(m.bias.data)
            out = q
            if act_cls is not None:
                a = act_cls(**self.kwargs)
                self.acts.append(a)
                out = nn.Sequential(a, q)
            return out.to(m.weight.device)
        if isinstance(m, nn.Conv2d) and "Conv2d" in self.replace_map:
            if self.is_first and not self.replace_first_layer:
                self.is_first = False
                return m
            act_cls, cls = self._split(self.replace_map["Conv2d"], nn.Conv2d)
            first = self.is_first
            kw = dict(self.kwargs)
            if first:  # the first layer is forced to 8 bits (replace_module.py:83-95)
                kw["nbits_w"], kw["nbits_a"] = 8, 8
            q = cls(m.in_channels, m.out_channels, m.kernel_size, m.stride, m.padding, m.dilation, groups=m.groups,
                    bias=m.bias is not None, **kw)
            self.convs.append(q)
            q.weight.data.copy_(m.weight.data)
            if m.bias is not None:
                q.bias.data.copy_(m.bias.data)
            out = q
            self.is_first = False
            if act_cls is not None:
                # the reference tests is_first again here, after clearing it, so the first layer's
                # activation quantiser keeps nbits_a (replace_module.py:104-109); kept as is
                a = act_cls(**self.kwargs)
                self.acts.append(a)
                out = nn.Sequential(a, q)
            return out.to(m.weight.device)
        return m
