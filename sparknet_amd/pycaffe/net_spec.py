"""Functional NetParameter builder with pycaffe's ``net_spec`` surface
(caffe/python/caffe/net_spec.py: ``layers`` / ``params`` pseudo-modules, ``NetSpec``,
``to_proto``).

    from sparknet_amd.pycaffe import layers as L, params as P, NetSpec
    n = NetSpec()
    n.data, n.label = L.DummyData(shape=[dict(dim=[64, 1, 28, 28]), dict(dim=[64, 1])], ntop=2)
    n.conv1 = L.Convolution(n.data, kernel_size=5, num_output=20, weight_filler=dict(type="xavier"))
    n.pool1 = L.Pooling(n.conv1, kernel_size=2, stride=2, pool=P.Pooling.MAX)
    n.loss = L.SoftmaxWithLoss(n.pool1, n.label)
    netparam = n.to_proto()

Keyword arguments become fields of the layer's ``<type>_param`` message when that message
has such a field, otherwise fields of the LayerParameter itself (``param``, ``include``,
``loss_weight``, ``transform_param``, ...).  Lists fill repeated fields, dicts fill
sub-messages.  Special keys: ``ntop`` (number of tops; 0 for sinks), ``in_place`` (top =
bottom).  Unnamed tops are named ``<Type><k>`` in creation order.
"""
from __future__ import annotations

from collections import Counter, OrderedDict

from .. import proto

__all__ = ["layers", "params", "NetSpec", "to_proto", "Top", "Function"]


def _param_field_of_type() -> dict:
    """Layer type name -> its ``*_param`` field name, from the LayerParameter descriptor
    (e.g. 'Convolution' -> 'convolution_param', 'LRN' -> 'lrn_param')."""
    out = {}
    for f in proto.LayerParameter.DESCRIPTOR.fields:
        if f.name.endswith("_param") and f.message_type is not None:
            tname = f.message_type.name
            if tname.endswith("Parameter"):
                out[tname[:-len("Parameter")]] = f.name
    return out


_TYPE_PARAM = _param_field_of_type()


def _assign(msg, name, val) -> None:
    field = getattr(msg, name)
    repeated = hasattr(field, "extend")
    if repeated and not isinstance(val, (list, tuple)):
        val = [val]
    if isinstance(val, (list, tuple)):
        if val and isinstance(val[0], dict):
            for item in val:
                sub = field.add()
                for k, v in item.items():
                    _assign(sub, k, v)
        else:
            field.extend(val)
    elif isinstance(val, dict):
        for k, v in val.items():
            _assign(field, k, v)
    else:
        setattr(msg, name, val)


class Top:
    """One output blob of a Function (a layer)."""

    def __init__(self, fn: "Function", n: int):
        self.fn, self.n = fn, n

    def to_proto(self):
        return to_proto(self)

    def _emit(self, layers, names, auto):
        self.fn._emit(layers, names, auto)


class Function:
    """A layer: type, input Tops and keyword parameters."""

    def __init__(self, type_name: str, inputs, params: dict):
        self.type_name = type_name
        self.inputs = list(inputs)
        params = dict(params)
        self.ntop = int(params.pop("ntop", 1))
        self.in_place = bool(params.pop("in_place", False))
        self.params = params
        self.tops = tuple(Top(self, i) for i in range(self.ntop))

    def _top_name(self, top, names, auto):
        if top not in names:
            auto[top.fn.type_name] += 1
            names[top] = f"{top.fn.type_name}{auto[top.fn.type_name]}"
        return names[top]

    def _name(self, names, auto):
        if self not in names:
            if self.ntop > 0:
                names[self] = self._top_name(self.tops[0], names, auto)
            else:
                auto[self.type_name] += 1
                names[self] = f"{self.type_name}{auto[self.type_name]}"
        return names[self]

    def _emit(self, layers, names, auto):
        if self in layers:
            return
        bottoms = []
        for inp in self.inputs:
            inp._emit(layers, names, auto)
            bottoms.append(layers[inp.fn].top[inp.n])
        lp = proto.LayerParameter(type=self.type_name)
        lp.bottom.extend(bottoms)
        if self.in_place:
            lp.top.extend(bottoms)
        else:
            lp.top.extend(self._top_name(t, names, auto) for t in self.tops)
        lp.name = self._name(names, auto)
        pfield = _TYPE_PARAM.get(self.type_name)
        for k, v in self.params.items():
            if k.endswith("param"):
                _assign(lp, k, v)
            elif pfield is not None and k in getattr(lp, pfield).DESCRIPTOR.fields_by_name:
                _assign(getattr(lp, pfield), k, v)
            else:
                _assign(lp, k, v)
        layers[self] = lp


def to_proto(*tops):
    """NetParameter with every layer needed to compute ``tops`` (auto-named blobs)."""
    layers, auto = OrderedDict(), Counter()
    for t in tops:
        t._emit(layers, {}, auto)
    net = proto.NetParameter()
    net.layer.extend(layers.values())
    return net


class NetSpec:
    """Assign Tops as attributes to name them; ``to_proto`` emits the named layers."""

    def __init__(self):
        super().__setattr__("tops", OrderedDict())

    def __setattr__(self, name, value):
        self.tops[name] = value

    def __getattr__(self, name):
        try:
            return self.tops[name]
        except KeyError as e:
            raise AttributeError(name) from e

    def __setitem__(self, name, value):
        self.tops[name] = value

    def __getitem__(self, name):
        return self.tops[name]

    def to_proto(self):
        names = {}
        for k, v in self.tops.items():
            if isinstance(v, Top):
                names[v] = k
            elif isinstance(v, Function):  # a zero-top layer assigned by name
                names[v] = k
        layers, auto = OrderedDict(), Counter()
        for v in self.tops.values():
            v._emit(layers, names, auto)
        net = proto.NetParameter()
        net.layer.extend(layers.values())
        return net


class _Layers:
    def __getattr__(self, type_name):
        def make(*inputs, **params):
            fn = Function(type_name, inputs, params)
            if fn.ntop == 0:
                return fn
            return fn.tops[0] if fn.ntop == 1 else fn.tops
        return make


class _Params:
    """``params.Pooling.MAX`` -> PoolingParameter.MAX (enum values by message type)."""

    def __getattr__(self, type_name):
        from ..proto.schema import message_class
        cls = message_class(type_name + "Parameter")

        class _Enum:
            def __getattr__(self, value):
                for et in cls.DESCRIPTOR.enum_types:
                    if value in et.values_by_name:
                        return et.values_by_name[value].number
                raise AttributeError(f"{type_name}Parameter has no enum value {value!r}")
        return _Enum()


layers = _Layers()
params = _Params()
