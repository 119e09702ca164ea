"""``graph.pbtxt`` and ``model.ckpt-N.meta`` for ``--log_dir`` (the files TF1's
``MonitoredTrainingSession`` writes beside its checkpoints, /root/reference/cifar10cnn.py:222).

The framework has no TF graph at run time, so these files describe the reference model as a TF1
graph would: the ``model_definition/...`` variables (VariableV2 + initializer + Assign + read), the
forward network of ``create_cnn`` (:94-147: Conv2D / BiasAdd / Relu / MaxPool / Reshape / MatMul /
Add) on an ``input_images`` placeholder, the loss (:150-157) and accuracy (:166-176), the
``global_step`` / ``Variable`` (generation_num) scalars, and a V2 ``save/`` subgraph (SaveV2,
RestoreV2, one Assign per variable, ``save/restore_all``) that the ``SaverDef`` names -- the pieces
``tf.train.import_meta_graph`` + ``Saver.restore`` use.  The training ops (gradients, SGD) are not
materialised: the step runs as HIP kernels.  Other models (ResNet-20) get the variables + saver.

Messages are built with the ``protobuf`` runtime from descriptors declared here with the field
numbers of TF's GraphDef / NodeDef / AttrValue / TensorProto / MetaGraphDef / SaverDef /
CollectionDef / VariableDef protos, so the binary ``.meta`` and the text ``graph.pbtxt`` use TF's
wire and text formats.  Parity with real TF output is unpinned (no TF in this environment):
``tests/test_metagraph.py`` checks the structure (every input resolves, every variable is saved and
restored, the SaverDef names exist) by parsing the files back.
"""
from __future__ import annotations

import functools
import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch

_F = None  # descriptor_pb2.FieldDescriptorProto (lazy import)

DT = {"float": 1, "double": 2, "int32": 3, "uint8": 4, "string": 7, "int64": 9, "bool": 10, "bfloat16": 14}
_TORCH_DT = {torch.float32: 1, torch.float64: 2, torch.int32: 3, torch.uint8: 4, torch.int64: 9, torch.bool: 10,
             torch.bfloat16: 14}


@functools.lru_cache(maxsize=1)
def _classes():
    """Message classes of the TF proto subset (package ``tensorflow``)."""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    F = descriptor_pb2.FieldDescriptorProto
    fdp = descriptor_pb2.FileDescriptorProto(name="dmlc/tf_metagraph_subset.proto", package="tensorflow",
                                             syntax="proto3")
    e = fdp.enum_type.add(name="DataType")
    for n, v in [("DT_INVALID", 0), ("DT_FLOAT", 1), ("DT_DOUBLE", 2), ("DT_INT32", 3), ("DT_UINT8", 4),
                 ("DT_INT16", 5), ("DT_INT8", 6), ("DT_STRING", 7), ("DT_COMPLEX64", 8), ("DT_INT64", 9),
                 ("DT_BOOL", 10), ("DT_BFLOAT16", 14), ("DT_HALF", 19)]:
        e.value.add(name=n, number=v)

    def fld(m, name, num, typ, label=F.LABEL_OPTIONAL, type_name=None, oneof=None):
        f = m.field.add(name=name, number=num, type=typ, label=label)
        if type_name:
            f.type_name = type_name
        if oneof is not None:
            f.oneof_index = oneof
        return f

    R = F.LABEL_REPEATED
    # TensorShapeProto
    m = fdp.message_type.add(name="TensorShapeProto")
    d = m.nested_type.add(name="Dim")
    fld(d, "size", 1, F.TYPE_INT64)
    fld(d, "name", 2, F.TYPE_STRING)
    fld(m, "dim", 2, F.TYPE_MESSAGE, R, ".tensorflow.TensorShapeProto.Dim")
    fld(m, "unknown_rank", 3, F.TYPE_BOOL)
    # TensorProto (the fields used here)
    m = fdp.message_type.add(name="TensorProto")
    fld(m, "dtype", 1, F.TYPE_ENUM, type_name=".tensorflow.DataType")
    fld(m, "tensor_shape", 2, F.TYPE_MESSAGE, type_name=".tensorflow.TensorShapeProto")
    fld(m, "version_number", 3, F.TYPE_INT32)
    fld(m, "tensor_content", 4, F.TYPE_BYTES)
    fld(m, "float_val", 5, F.TYPE_FLOAT, R)
    fld(m, "double_val", 6, F.TYPE_DOUBLE, R)
    fld(m, "int_val", 7, F.TYPE_INT32, R)
    fld(m, "string_val", 8, F.TYPE_BYTES, R)
    fld(m, "int64_val", 10, F.TYPE_INT64, R)
    fld(m, "bool_val", 11, F.TYPE_BOOL, R)
    # AttrValue
    m = fdp.message_type.add(name="AttrValue")
    lv = m.nested_type.add(name="ListValue")
    fld(lv, "s", 2, F.TYPE_BYTES, R)
    fld(lv, "i", 3, F.TYPE_INT64, R)
    fld(lv, "f", 4, F.TYPE_FLOAT, R)
    fld(lv, "b", 5, F.TYPE_BOOL, R)
    fld(lv, "type", 6, F.TYPE_ENUM, R, ".tensorflow.DataType")
    fld(lv, "shape", 7, F.TYPE_MESSAGE, R, ".tensorflow.TensorShapeProto")
    fld(lv, "tensor", 8, F.TYPE_MESSAGE, R, ".tensorflow.TensorProto")
    m.oneof_decl.add(name="value")
    fld(m, "list", 1, F.TYPE_MESSAGE, type_name=".tensorflow.AttrValue.ListValue", oneof=0)
    fld(m, "s", 2, F.TYPE_BYTES, oneof=0)
    fld(m, "i", 3, F.TYPE_INT64, oneof=0)
    fld(m, "f", 4, F.TYPE_FLOAT, oneof=0)
    fld(m, "b", 5, F.TYPE_BOOL, oneof=0)
    fld(m, "type", 6, F.TYPE_ENUM, type_name=".tensorflow.DataType", oneof=0)
    fld(m, "shape", 7, F.TYPE_MESSAGE, type_name=".tensorflow.TensorShapeProto", oneof=0)
    fld(m, "tensor", 8, F.TYPE_MESSAGE, type_name=".tensorflow.TensorProto", oneof=0)
    fld(m, "placeholder", 9, F.TYPE_STRING, oneof=0)

    def map_entry(parent, name, value_type, value_type_name=None):
        ent = parent.nested_type.add(name=name)
        ent.options.map_entry = True
        fld(ent, "key", 1, F.TYPE_STRING)
        fld(ent, "value", 2, value_type, type_name=value_type_name)
        return ent

    # NodeDef
    m = fdp.message_type.add(name="NodeDef")
    fld(m, "name", 1, F.TYPE_STRING)
    fld(m, "op", 2, F.TYPE_STRING)
    fld(m, "input", 3, F.TYPE_STRING, R)
    fld(m, "device", 4, F.TYPE_STRING)
    map_entry(m, "AttrEntry", F.TYPE_MESSAGE, ".tensorflow.AttrValue")
    fld(m, "attr", 5, F.TYPE_MESSAGE, R, ".tensorflow.NodeDef.AttrEntry")
    # VersionDef, GraphDef
    m = fdp.message_type.add(name="VersionDef")
    fld(m, "producer", 1, F.TYPE_INT32)
    fld(m, "min_consumer", 2, F.TYPE_INT32)
    fld(m, "bad_consumers", 3, F.TYPE_INT32, R)
    m = fdp.message_type.add(name="GraphDef")
    fld(m, "node", 1, F.TYPE_MESSAGE, R, ".tensorflow.NodeDef")
    fld(m, "versions", 4, F.TYPE_MESSAGE, type_name=".tensorflow.VersionDef")
    # SaverDef
    m = fdp.message_type.add(name="SaverDef")
    ev = m.enum_type.add(name="CheckpointFormatVersion")
    for n, v in [("LEGACY", 0), ("V1", 1), ("V2", 2)]:
        ev.value.add(name=n, number=v)
    fld(m, "filename_tensor_name", 1, F.TYPE_STRING)
    fld(m, "save_tensor_name", 2, F.TYPE_STRING)
    fld(m, "restore_op_name", 3, F.TYPE_STRING)
    fld(m, "max_to_keep", 4, F.TYPE_INT32)
    fld(m, "sharded", 5, F.TYPE_BOOL)
    fld(m, "keep_checkpoint_every_n_hours", 6, F.TYPE_FLOAT)
    fld(m, "version", 7, F.TYPE_ENUM, type_name=".tensorflow.SaverDef.CheckpointFormatVersion")
    # CollectionDef
    m = fdp.message_type.add(name="CollectionDef")
    for nm, num, typ in (("NodeList", 1, F.TYPE_STRING), ("BytesList", 2, F.TYPE_BYTES),
                         ("Int64List", 3, F.TYPE_INT64), ("FloatList", 4, F.TYPE_FLOAT)):
        sub = m.nested_type.add(name=nm)
        fld(sub, "value", 1, typ, R)
    m.oneof_decl.add(name="kind")
    fld(m, "node_list", 1, F.TYPE_MESSAGE, type_name=".tensorflow.CollectionDef.NodeList", oneof=0)
    fld(m, "bytes_list", 2, F.TYPE_MESSAGE, type_name=".tensorflow.CollectionDef.BytesList", oneof=0)
    fld(m, "int64_list", 3, F.TYPE_MESSAGE, type_name=".tensorflow.CollectionDef.Int64List", oneof=0)
    fld(m, "float_list", 4, F.TYPE_MESSAGE, type_name=".tensorflow.CollectionDef.FloatList", oneof=0)
    # VariableDef
    m = fdp.message_type.add(name="VariableDef")
    fld(m, "variable_name", 1, F.TYPE_STRING)
    fld(m, "initializer_name", 2, F.TYPE_STRING)
    fld(m, "snapshot_name", 3, F.TYPE_STRING)
    fld(m, "is_resource", 5, F.TYPE_BOOL)
    fld(m, "initial_value_name", 6, F.TYPE_STRING)
    fld(m, "trainable", 7, F.TYPE_BOOL)
    # MetaGraphDef
    m = fdp.message_type.add(name="MetaGraphDef")
    mi = m.nested_type.add(name="MetaInfoDef")
    fld(mi, "meta_graph_version", 1, F.TYPE_STRING)
    fld(mi, "tags", 4, F.TYPE_STRING, R)
    fld(mi, "tensorflow_version", 5, F.TYPE_STRING)
    fld(mi, "tensorflow_git_version", 6, F.TYPE_STRING)
    fld(mi, "stripped_default_attrs", 7, F.TYPE_BOOL)
    map_entry(m, "CollectionDefEntry", F.TYPE_MESSAGE, ".tensorflow.CollectionDef")
    fld(m, "meta_info_def", 1, F.TYPE_MESSAGE, type_name=".tensorflow.MetaGraphDef.MetaInfoDef")
    fld(m, "graph_def", 2, F.TYPE_MESSAGE, type_name=".tensorflow.GraphDef")
    fld(m, "saver_def", 3, F.TYPE_MESSAGE, type_name=".tensorflow.SaverDef")
    fld(m, "collection_def", 4, F.TYPE_MESSAGE, R, ".tensorflow.MetaGraphDef.CollectionDefEntry")

    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    names = ["TensorShapeProto", "TensorProto", "AttrValue", "NodeDef", "GraphDef", "SaverDef", "CollectionDef",
             "VariableDef", "MetaGraphDef"]
    return {n: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"tensorflow.{n}")) for n in names}


# ------------------------------------------------------------------------------------------------
class _Graph:
    """A GraphDef under construction (TF1 naming: scope/op, then scope/op_1, ...)."""

    def __init__(self):
        C = _classes()
        self.C = C
        self.g = C["GraphDef"]()
        self.g.versions.producer = 27        # a TF 1.x-era GraphDef producer version
        self.names = set()

    def unique(self, name: str) -> str:
        if name not in self.names:
            return name
        i = 1
        while f"{name}_{i}" in self.names:
            i += 1
        return f"{name}_{i}"

    def node(self, name: str, op: str, inputs: Sequence[str] = (), **attrs) -> str:
        name = self.unique(name)
        self.names.add(name)
        n = self.g.node.add(name=name, op=op)
        n.input.extend(inputs)
        for k, v in attrs.items():
            _set_attr(n.attr[k], v, self.C)
        return name

    # helpers ------------------------------------------------------------------------------------
    def const(self, name, value, dtype="float", shape: Optional[Sequence[int]] = None) -> str:
        t = _tensor(value, dtype, shape, self.C)
        return self.node(name, "Const", dtype=("type", DT[dtype]), value=("tensor", t))


def _shape_proto(shape, C):
    s = C["TensorShapeProto"]()
    if shape is None:
        s.unknown_rank = True
    else:
        for d in shape:
            s.dim.add(size=int(d))
    return s


def _tensor(value, dtype, shape, C):
    t = C["TensorProto"](dtype=DT[dtype])
    vals = value if isinstance(value, (list, tuple)) else [value]
    t.tensor_shape.CopyFrom(_shape_proto(shape if shape is not None else ([] if not isinstance(value, (list, tuple))
                                                                        else [len(vals)]), C))
    if dtype == "float":
        t.float_val.extend(float(v) for v in vals)
    elif dtype == "int32":
        t.int_val.extend(int(v) for v in vals)
    elif dtype == "int64":
        t.int64_val.extend(int(v) for v in vals)
    elif dtype == "string":
        t.string_val.extend(v.encode() if isinstance(v, str) else v for v in vals)
    elif dtype == "bool":
        t.bool_val.extend(bool(v) for v in vals)
    else:
        raise ValueError(dtype)
    return t


def _set_attr(a, v, C):
    kind, val = v
    if kind == "type":
        a.type = val
    elif kind == "shape":
        a.shape.CopyFrom(_shape_proto(val, C))
    elif kind == "tensor":
        a.tensor.CopyFrom(val)
    elif kind == "s":
        a.s = val.encode() if isinstance(val, str) else val
    elif kind == "i":
        a.i = int(val)
    elif kind == "f":
        a.f = float(val)
    elif kind == "b":
        a.b = bool(val)
    elif kind == "list_i":
        a.list.i.extend(int(x) for x in val)
    elif kind == "list_type":
        a.list.type.extend(val)
    elif kind == "list_s":
        a.list.s.extend(x.encode() if isinstance(x, str) else x for x in val)
    else:
        raise ValueError(kind)


def _variable(G: _Graph, name: str, shape: Sequence[int], dtype: str, init: Tuple[str, float]) -> Dict[str, str]:
    """VariableV2 + initializer + Assign + read, TF1 ``get_variable`` naming."""
    var = G.node(name, "VariableV2", shape=("shape", list(shape)), dtype=("type", DT[dtype]),
                 container=("s", ""), shared_name=("s", ""))
    kind, val = init
    if kind == "trunc_normal":
        shp = G.const(f"{name}/Initializer/truncated_normal/shape", list(shape), "int32", [len(shape)])
        mean = G.const(f"{name}/Initializer/truncated_normal/mean", 0.0)
        std = G.const(f"{name}/Initializer/truncated_normal/stddev", val)
        tn = G.node(f"{name}/Initializer/truncated_normal/TruncatedNormal", "TruncatedNormal", [shp],
                    T=("type", DT["int32"]), dtype=("type", DT[dtype]), seed=("i", 0), seed2=("i", 0))
        mul = G.node(f"{name}/Initializer/truncated_normal/mul", "Mul", [tn, std], T=("type", DT[dtype]))
        initv = G.node(f"{name}/Initializer/truncated_normal", "Add", [mul, mean], T=("type", DT[dtype]))
    else:    # constant fill (TF broadcasts a single value over the Const's shape)
        initv = G.const(f"{name}/Initializer/Const", val if dtype != "int32" and dtype != "int64" else int(val),
                        dtype, list(shape))
    assign = G.node(f"{name}/Assign", "Assign", [var, initv], T=("type", DT[dtype]), validate_shape=("b", True),
                    use_locking=("b", True), _class=("list_s", [f"loc:@{name}"]))
    read = G.node(f"{name}/read", "Identity", [var], T=("type", DT[dtype]), _class=("list_s", [f"loc:@{name}"]))
    return {"var": var, "initial": initv, "assign": assign, "read": read, "dtype": dtype, "shape": list(shape)}


def _cnn_forward(G: _Graph, v: Dict[str, Dict[str, str]], x: str, batch: int, relu_logits: bool,
                 scope: str = "model_definition") -> str:
    """create_cnn (cifar10cnn.py:94-147) on input tensor ``x`` (NHWC float)."""
    f = ("type", DT["float"])

    def conv(name, inp, k, b):
        c = G.node(f"{scope}/{name}/Conv2D", "Conv2D", [inp, v[k]["read"]], T=f, strides=("list_i", [1, 1, 1, 1]),
                   padding=("s", "SAME"), data_format=("s", "NHWC"), use_cudnn_on_gpu=("b", True),
                   dilations=("list_i", [1, 1, 1, 1]))
        ba = G.node(f"{scope}/{name}/BiasAdd", "BiasAdd", [c, v[b]["read"]], T=f, data_format=("s", "NHWC"))
        return G.node(f"{scope}/{name}/Relu", "Relu", [ba], T=f)

    def pool(name, inp):
        return G.node(f"{scope}/{name}", "MaxPool", [inp], T=f, ksize=("list_i", [1, 3, 3, 1]),
                      strides=("list_i", [1, 2, 2, 1]), padding=("s", "SAME"), data_format=("s", "NHWC"))

    def full(name, inp, w, b, relu=True):
        mm = G.node(f"{scope}/{name}/MatMul", "MatMul", [inp, v[w]["read"]], T=f, transpose_a=("b", False),
                    transpose_b=("b", False))
        add = G.node(f"{scope}/{name}/Add", "Add", [mm, v[b]["read"]], T=f)
        return G.node(f"{scope}/{name}/Relu", "Relu", [add], T=f) if relu else add

    p = "model_definition/"
    h = conv("conv1", x, p + "conv1/conv1_kernel", p + "conv1/conv1_bias")
    h = pool("pool1", h)
    h = conv("conv2", h, p + "conv2/conv2_kernel", p + "conv2/conv2_bias")
    h = pool("pool2", h)
    shp = G.const(f"{scope}/Reshape/shape", [batch, -1], "int32", [2])
    h = G.node(f"{scope}/Reshape", "Reshape", [h, shp], T=f, Tshape=("type", DT["int32"]))
    h = full("full1", h, p + "full1/full_weight_1", p + "full1/full_bias_1")
    h = full("full2", h, p + "full2/full_weight_2", p + "full2/full_bias_2")
    return full("full3", h, p + "full3/full_weight_3", p + "full3/full_bias_3", relu=relu_logits)


def _var_init(name: str) -> Tuple[str, float]:
    if name.endswith("_kernel") or "full_weight" in name or name.endswith("/weights"):
        return ("trunc_normal", 0.05)
    if name in ("global_step", "Variable"):
        return ("const", 0)
    if name.endswith("/gamma") or name.endswith("moving_variance"):
        return ("const", 1.0)
    if name.endswith("/beta") or name.endswith("moving_mean"):
        return ("const", 0.0)
    return ("const", 0.1)


def build_meta_graph(tensors: Dict[str, torch.Tensor], model: str = "cifar_cnn", batch: int = 128,
                     crop: int = 24, relu_logits: bool = True, max_to_keep: int = 5):
    """MetaGraphDef message for a checkpoint whose variables are ``tensors`` (name -> tensor)."""
    C = _classes()
    G = _Graph()
    names = sorted(tensors)                         # SaveV2 / RestoreV2 list variables in name order
    v = {}
    for n in names:
        t = tensors[n]
        dt = {1: "float", 2: "double", 3: "int32", 9: "int64", 4: "uint8", 10: "bool", 14: "bfloat16"}[_TORCH_DT[t.dtype]]
        v[n] = _variable(G, n, list(t.shape), dt, _var_init(n))
    outputs = {}
    if model in ("cifar_cnn", "cnn", "cifar10_cnn"):
        x = G.node("input_images", "Placeholder", dtype=("type", DT["float"]),
                   shape=("shape", [batch, crop, crop, 3]))
        y = G.node("input_labels", "Placeholder", dtype=("type", DT["int32"]), shape=("shape", [batch]))
        logits = _cnn_forward(G, v, x, batch, relu_logits)
        xent = G.node("SparseSoftmaxCrossEntropyWithLogits/SparseSoftmaxCrossEntropyWithLogits",
                      "SparseSoftmaxCrossEntropyWithLogits", [logits, y], T=("type", DT["float"]),
                      Tlabels=("type", DT["int32"]))
        axis = G.const("Const", [0], "int32", [1])
        loss = G.node("cross_entropy", "Mean", [xent, axis], T=("type", DT["float"]), Tidx=("type", DT["int32"]),
                      keep_dims=("b", False))
        dim = G.const("ArgMax/dimension", 1, "int32")
        am = G.node("ArgMax", "ArgMax", [logits, dim], T=("type", DT["float"]), Tidx=("type", DT["int32"]),
                    output_type=("type", DT["int64"]))
        amc = G.node("Cast", "Cast", [am], SrcT=("type", DT["int64"]), DstT=("type", DT["int32"]),
                     Truncate=("b", False))
        eq = G.node("Equal", "Equal", [amc, y], T=("type", DT["int32"]))
        eqf = G.node("Cast_1", "Cast", [eq], SrcT=("type", DT["bool"]), DstT=("type", DT["float"]),
                     Truncate=("b", False))
        ax2 = G.const("Const_1", [0], "int32", [1])
        acc = G.node("accuracy", "Mean", [eqf, ax2], T=("type", DT["float"]), Tidx=("type", DT["int32"]),
                     keep_dims=("b", False))
        outputs = {"logits": logits, "loss": loss, "accuracy": acc}
    # ---- saver (V2, one shard) --------------------------------------------------------------------
    fn_in = G.const("save/filename/input", "model", "string")
    fn = G.node("save/filename", "PlaceholderWithDefault", [fn_in], dtype=("type", DT["string"]),
                shape=("shape", []))
    sc = G.node("save/Const", "PlaceholderWithDefault", [fn], dtype=("type", DT["string"]), shape=("shape", []))
    tn = G.const("save/SaveV2/tensor_names", names, "string", [len(names)])
    ss = G.const("save/SaveV2/shape_and_slices", [""] * len(names), "string", [len(names)])
    dts = [DT[v[n]["dtype"]] for n in names]
    save = G.node("save/SaveV2", "SaveV2", [sc, tn, ss] + [v[n]["var"] for n in names], dtypes=("list_type", dts))
    cd = G.node("save/control_dependency", "Identity", [sc, "^" + save], T=("type", DT["string"]),
                _class=("list_s", ["loc:@save/Const"]))
    rtn = G.const("save/RestoreV2/tensor_names", names, "string", [len(names)])
    rss = G.const("save/RestoreV2/shape_and_slices", [""] * len(names), "string", [len(names)])
    rst = G.node("save/RestoreV2", "RestoreV2", [sc, rtn, rss], dtypes=("list_type", dts))
    assigns = []
    for i, n in enumerate(names):
        assigns.append(G.node("save/Assign", "Assign", [v[n]["var"], f"{rst}:{i}" if i else rst],
                              T=("type", DT[v[n]["dtype"]]), validate_shape=("b", True), use_locking=("b", True),
                              _class=("list_s", [f"loc:@{n}"])))
    restore_all = G.node("save/restore_all", "NoOp", ["^" + a for a in assigns])
    init = G.node("init", "NoOp", ["^" + v[n]["assign"] for n in names])
    # ---- MetaGraphDef -----------------------------------------------------------------------------
    mg = C["MetaGraphDef"]()
    mg.meta_info_def.meta_graph_version = "v1"
    mg.meta_info_def.tensorflow_git_version = "dmlc (MI355X HIP engine; graph for import_meta_graph)"
    mg.graph_def.CopyFrom(G.g)
    sd = mg.saver_def
    sd.filename_tensor_name = f"{sc}:0"
    sd.save_tensor_name = f"{cd}:0"
    sd.restore_op_name = restore_all
    sd.max_to_keep = int(max_to_keep)
    sd.sharded = False
    sd.keep_checkpoint_every_n_hours = 10000.0
    sd.version = 2

    def vdef(n, trainable):
        d = C["VariableDef"](variable_name=f"{v[n]['var']}:0", initializer_name=v[n]["assign"],
                             snapshot_name=f"{v[n]['read']}:0", initial_value_name=f"{v[n]['initial']}:0",
                             trainable=trainable)
        return d.SerializeToString()

    trainable = [n for n in names if n not in ("global_step", "Variable") and "moving_" not in n]
    mg.collection_def["variables"].bytes_list.value.extend(vdef(n, n in trainable) for n in names)
    mg.collection_def["trainable_variables"].bytes_list.value.extend(vdef(n, True) for n in trainable)
    if "global_step" in v:
        mg.collection_def["global_step"].bytes_list.value.append(vdef("global_step", False))
    for key, t in outputs.items():
        mg.collection_def[key].node_list.value.append(f"{t}:0")
    mg.collection_def["init_op"].node_list.value.append(init)
    return mg


def write_graph_pbtxt(log_dir: str, meta) -> str:
    """``<log_dir>/graph.pbtxt``: the GraphDef in protobuf text format (what TF's hook writes)."""
    from google.protobuf import text_format
    path = os.path.join(log_dir, "graph.pbtxt")
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        f.write(text_format.MessageToString(meta.graph_def))
    os.replace(tmp, path)
    return path


def write_meta(prefix: str, meta) -> str:
    """``<prefix>.meta``: the binary MetaGraphDef."""
    path = prefix + ".meta"
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(meta.SerializeToString())
    os.replace(tmp, path)
    return path


def read_meta(path: str):
    C = _classes()
    m = C["MetaGraphDef"]()
    with open(path, "rb") as f:
        m.ParseFromString(f.read())
    return m


def variable_defs(meta, collection: str = "variables") -> List:
    C = _classes()
    out = []
    for b in meta.collection_def[collection].bytes_list.value:
        d = C["VariableDef"]()
        d.ParseFromString(b)
        out.append(d)
    return out
