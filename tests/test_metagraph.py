"""graph.pbtxt / model.ckpt-N.meta (utils/metagraph.py): the files TF1's MonitoredTrainingSession
writes beside its checkpoints (/root/reference/cifar10cnn.py:222).  No TF here, so parity with TF's
own output is unpinned; these tests check the structure by parsing the files back: every node input
resolves, the SaverDef names exist, every checkpoint variable is saved, restored and listed in the
variables collection, and the forward graph follows create_cnn."""
import os

import torch

from dmlc import checkpoint as CK
from dmlc.models import cifar_cnn as M
from dmlc.utils import metagraph as MG


def _tensors():
    return CK.model_tensors(M.init_flat_params(torch.Generator().manual_seed(0)), 7, 0)


def _node_map(g):
    return {n.name: n for n in g.node}


def test_graph_is_closed_and_saver_is_complete():
    t = _tensors()
    mg = MG.build_meta_graph(t, batch=128, crop=24)
    mg2 = MG._classes()["MetaGraphDef"]()
    mg2.ParseFromString(mg.SerializeToString())            # binary round trip
    nodes = _node_map(mg2.graph_def)
    assert len(nodes) == len(mg2.graph_def.node)            # unique names
    for n in mg2.graph_def.node:
        for i in n.input:
            src = i.lstrip("^").split(":")[0]
            assert src in nodes, (n.name, i)
    sd = mg2.saver_def
    assert sd.filename_tensor_name.split(":")[0] in nodes
    assert sd.save_tensor_name.split(":")[0] in nodes
    assert nodes[sd.restore_op_name].op == "NoOp" and sd.version == 2
    names = sorted(t)
    save = nodes["save/SaveV2"]
    assert list(save.attr["dtypes"].list.type) == [1 if t[n].dtype == torch.float32 else
                                                   (9 if t[n].dtype == torch.int64 else 3) for n in names]
    assert [s.decode() for s in nodes["save/SaveV2/tensor_names"].attr["value"].tensor.string_val] == names
    assert [s.decode() for s in nodes["save/RestoreV2/tensor_names"].attr["value"].tensor.string_val] == names
    restored = {nodes[a.lstrip("^")].input[0] for a in nodes[sd.restore_op_name].input}
    assert restored == set(names)
    for n in names:                                          # VariableV2 with the checkpoint's shape
        v = nodes[n]
        assert v.op == "VariableV2"
        assert [d.size for d in v.attr["shape"].shape.dim] == list(t[n].shape)
    vd = MG.variable_defs(mg2)
    assert sorted(d.variable_name[:-2] for d in vd) == names
    assert all(d.snapshot_name.split(":")[0] in nodes and d.initializer_name in nodes for d in vd)
    trainable = {d.variable_name[:-2] for d in MG.variable_defs(mg2, "trainable_variables")}
    assert trainable == {s.name for s in M.PARAM_SPECS}


def test_forward_graph_follows_create_cnn():
    mg = MG.build_meta_graph(_tensors(), batch=64, crop=24, relu_logits=True)
    nodes = _node_map(mg.graph_def)
    ops = [n.op for n in mg.graph_def.node]
    assert ops.count("Conv2D") == 2 and ops.count("MaxPool") == 2 and ops.count("MatMul") == 3
    c1 = nodes["model_definition/conv1/Conv2D"]
    assert c1.attr["padding"].s == b"SAME" and list(c1.attr["strides"].list.i) == [1, 1, 1, 1]
    assert c1.input == ["input_images", "model_definition/conv1/conv1_kernel/read"]
    p1 = nodes["model_definition/pool1"]
    assert list(p1.attr["ksize"].list.i) == [1, 3, 3, 1] and list(p1.attr["strides"].list.i) == [1, 2, 2, 1]
    assert [d.size for d in nodes["input_images"].attr["shape"].shape.dim] == [64, 24, 24, 3]
    assert nodes["model_definition/full3/Relu"].op == "Relu"              # ReLU on the logits (D4)
    assert mg.collection_def["logits"].node_list.value == ["model_definition/full3/Relu:0"]
    assert nodes["cross_entropy"].op == "Mean"
    no_relu = MG.build_meta_graph(_tensors(), relu_logits=False)
    assert "model_definition/full3/Relu" not in _node_map(no_relu.graph_def)


def test_checkpoint_manager_writes_pbtxt_and_meta(tmp_path):
    from google.protobuf import text_format
    mgr = CK.CheckpointManager(str(tmp_path), max_to_keep=2, secs=0,
                               graph_info=dict(model="cifar_cnn", batch=128, crop=24, relu_logits=True))
    t = _tensors()
    for step in (1, 2, 3):
        mgr.save(step, t)
    assert os.path.exists(tmp_path / "graph.pbtxt")
    assert not os.path.exists(tmp_path / "model.ckpt-1.meta")                # rotated with its checkpoint
    meta = MG.read_meta(str(tmp_path / "model.ckpt-3.meta"))
    g = MG._classes()["GraphDef"]()
    text_format.Parse(open(tmp_path / "graph.pbtxt").read(), g)
    assert g == meta.graph_def
    assert CK.latest_checkpoint(str(tmp_path)).endswith("model.ckpt-3")


def test_resnet_checkpoint_gets_variables_and_saver():
    from dmlc.models import resnet as R
    flat, state = R.init_flat_params(torch.Generator().manual_seed(0))
    d = {s.name: flat[s.offset:s.offset + s.numel].view(s.shape) for s in R.PARAM_SPECS}
    d.update({s.name: state[s.offset:s.offset + s.numel].view(s.shape) for s in R.STATE_SPECS})
    d["global_step"] = torch.tensor(3, dtype=torch.int64)
    mg = MG.build_meta_graph(d, model="resnet20")
    nodes = _node_map(mg.graph_def)
    assert "input_images" not in nodes and len(MG.variable_defs(mg)) == len(d)
