"""TensorFlow graph artefacts without TensorFlow: ``saved_model.pb`` and the Saver's
``model.ckpt-<step>.meta``, hand-encoded in protobuf wire format.

Reference: ``export_model`` (`test_dist.py:511-532`) writes a SavedModel with tag
``serve`` and the signature ``intel_unet_brats_model`` {``image`` ->
``prediction``} that ``sanity_check_trained_model.py:38-41`` loads by tensor name
(``Placeholder:0`` -> ``Mask/Sigmoid:0``); the Supervisor's Saver writes a
``.meta`` MetaGraphDef next to every checkpoint (`test_dist.py:269-271,446,490`).

Here the GraphDef is the inference graph of the UNet spec in TF 1.x op vocabulary
(NHWC / NDHWC): ``Placeholder`` -> per layer ``VariableV2`` + ``Identity`` reads,
``Conv2D``/``Conv3D`` + ``BiasAdd`` + ``Relu`` (BatchNorm / GroupNorm [EXT] as
``FusedBatchNorm`` inference / a ``GroupNorm`` placeholder op), ``MaxPool``,
``Conv2DBackpropInput`` for the transposed convs (output size from ``Shape`` of
the input), ``ResizeNearestNeighbor`` for the 2D upsampling variant (3D: the
nearest upsample as ``Reshape`` -> ``Tile`` -> ``Reshape``, TF 1.x has no 3D resize
op), ``ConcatV2`` for the skips, ``Mask/Sigmoid`` at the end, plus the V2 Saver
subgraph (``save/Const``, ``save/SaveV2``, ``save/RestoreV2``, ``save/Assign_*``,
``save/restore_all``) that a SaverDef points at.  Every variable has the nodes its
VariableDef names: ``<v>/Initializer/zeros`` -> ``<v>/Assign`` (initializer) and
``<v>/read`` (snapshot).  Dropout is not in the exported graph (inference mode,
SURVEY.md Q9).

:func:`read_saved_model` parses the file back (tag, signature, GraphDef nodes and
the VariableV2 shapes) and :func:`spec_from_graph` recovers the UNet architecture
from the graph alone -- the exported ``saved_model.pb`` is the artefact
``inference.load_saved_model`` consumes.

Format parity is UNPINNED: TensorFlow is not installed, so the bytes are checked
structurally (field numbers, names, shapes, signature) by tests/test_io_formats.py,
not by loading them in TF.
"""

import os
from typing import Dict, List, Optional, Sequence, Tuple

from .tf_bundle import _fbytes, _field, _fv

DT_FLOAT, DT_INT32, DT_STRING, DT_INT64 = 1, 3, 7, 9
TF_VERSION = "1.4.0"


# ------------------------------------------------------------------ small encoders
def _s(num, text: str) -> bytes:
    return _fbytes(num, text.encode())


def _shape(dims: Optional[Sequence[int]]) -> bytes:
    """TensorShapeProto (dims None = unknown rank)."""
    if dims is None:
        return _fv(3, 1)
    return b"".join(_fbytes(2, _fv(1, int(d))) for d in dims)


def _a_type(t: int) -> bytes:          # AttrValue.type
    return _fv(6, t)


def _a_shape(dims) -> bytes:           # AttrValue.shape
    return _fbytes(7, _shape(dims))


def _a_s(text: str) -> bytes:          # AttrValue.s
    return _fbytes(2, text.encode())


def _a_b(v: bool) -> bytes:            # AttrValue.b
    return _fv(5, int(v))


def _a_i(v: int) -> bytes:             # AttrValue.i
    return _fv(3, int(v))


def _a_f(v: float) -> bytes:           # AttrValue.f
    import struct
    return _field(4, 5, struct.pack("<f", float(v)))


def _a_ints(vals) -> bytes:            # AttrValue.list.i (packed)
    from .tf_bundle import _varint
    packed = b"".join(_varint(int(v)) for v in vals)
    return _fbytes(1, _fbytes(3, packed))


def _a_types(vals) -> bytes:           # AttrValue.list.type (packed)
    from .tf_bundle import _varint
    return _fbytes(1, _fbytes(6, b"".join(_varint(int(v)) for v in vals)))


def _tensor_int32(vals, shape) -> bytes:
    """TensorProto: dtype, tensor_shape, int_val (packed)."""
    from .tf_bundle import _varint
    return _fv(1, DT_INT32) + _fbytes(2, _shape(shape)) + _fbytes(7, b"".join(_varint(int(v)) for v in vals))


def _tensor_strings(vals: List[str], shape) -> bytes:
    return _fv(1, DT_STRING) + _fbytes(2, _shape(shape)) + b"".join(_fbytes(8, v.encode()) for v in vals)


def _a_tensor(t: bytes) -> bytes:      # AttrValue.tensor
    return _fbytes(8, t)


def _map_entry(key: str, value: bytes) -> bytes:
    return _s(1, key) + _fbytes(2, value)


class _Graph:
    """GraphDef builder: NodeDef {name 1, op 2, input 3, device 4, attr 5 (map)}."""

    def __init__(self):
        self.nodes: List[bytes] = []
        self.names: List[str] = []

    def node(self, name: str, op: str, inputs: Sequence[str] = (), **attrs) -> str:
        b = _s(1, name) + _s(2, op) + b"".join(_s(3, i) for i in inputs)
        for k in sorted(attrs):
            b += _fbytes(5, _map_entry(k, attrs[k]))
        self.nodes.append(b)
        self.names.append(name)
        return name

    def const_i32(self, name: str, vals, shape) -> str:
        return self.node(name, "Const", dtype=_a_type(DT_INT32), value=_a_tensor(_tensor_int32(vals, shape)))

    def encode(self) -> bytes:
        # GraphDef: node 1 (repeated), versions 4 (VersionDef producer 1 = 24, TF 1.4)
        return b"".join(_fbytes(1, n) for n in self.nodes) + _fbytes(4, _fv(1, 24))


def _tensor_zero(dtype: int, shape) -> bytes:
    """TensorProto of `shape` filled with 0 (one value; TF repeats the last value)."""
    import struct
    val = _fbytes(10, b"\x00") if dtype == DT_INT64 else _fbytes(5, struct.pack("<f", 0.0))
    return _fv(1, dtype) + _fbytes(2, _shape(shape)) + val


def _variable(g: _Graph, name: str, shape, dtype: int = DT_FLOAT) -> str:
    """VariableV2 + the nodes its VariableDef names: <v>/Initializer/zeros -> <v>/Assign
    (initializer_name) and <v>/read (snapshot_name).  Returns the snapshot."""
    loc = _fbytes(1, _fbytes(2, ("loc:@" + name).encode()))
    g.node(name, "VariableV2", shape=_a_shape(shape), dtype=_a_type(dtype), container=_a_s(""),
           shared_name=_a_s(""))
    z = g.node(name + "/Initializer/zeros", "Const", dtype=_a_type(dtype), value=_a_tensor(_tensor_zero(dtype, shape)),
               _class=loc)
    g.node(name + "/Assign", "Assign", [name, z], T=_a_type(dtype), validate_shape=_a_b(True),
           use_locking=_a_b(True), _class=loc)
    return g.node(name + "/read", "Identity", [name], T=_a_type(dtype), _class=loc)


def build_graph(spec, img_size: int, extra_vars: Sequence[Tuple[str, Tuple[int, ...]]] = ()) -> Tuple[_Graph, List[Tuple[str, Tuple[int, ...]]]]:
    """Inference graph of `spec` + the Saver subgraph over every variable of the
    checkpoint (the model's and `extra_vars`, e.g. Adam slots / global_step)."""
    g = _Graph()
    dims = spec.dims
    conv_op = "Conv3D" if dims == 3 else "Conv2D"
    pool_op = "MaxPool3D" if dims == 3 else "MaxPool"
    ones = [1] * (dims + 2)
    x_shape = [-1] + [img_size] * dims + [spec.in_channels]
    cur = g.node("Placeholder", "Placeholder", dtype=_a_type(DT_FLOAT), shape=_a_shape(x_shape))
    outs: Dict[str, str] = {}
    pending_up = None
    variables = list(spec.variables())
    for l in spec.layers:
        if l.kind in ("conv", "mask"):
            if l.skip_from is not None:
                up = pending_up if pending_up is not None else cur
                axis = g.const_i32("concatenate_%s/concat/axis" % l.name, [dims + 1], [])
                cur = g.node("concatenate_%s/concat" % l.name, "ConcatV2", [up, outs[l.skip_from], axis],
                             T=_a_type(DT_FLOAT), N=_a_i(2), Tidx=_a_type(DT_INT32))
                pending_up = None
            k = _variable(g, l.name + "/kernel", l.kernel_shape(dims))
            b = _variable(g, l.name + "/bias", (l.cout,))
            attrs = dict(T=_a_type(DT_FLOAT), strides=_a_ints(ones), padding=_a_s("SAME"),
                         data_format=_a_s("NDHWC" if dims == 3 else "NHWC"))
            if dims == 2:
                attrs.update(use_cudnn_on_gpu=_a_b(True), dilations=_a_ints(ones))
            y = g.node(l.name + "/convolution", conv_op, [cur, k], **attrs)
            y = g.node(l.name + "/BiasAdd", "BiasAdd", [y, b], T=_a_type(DT_FLOAT),
                       data_format=_a_s("NHWC"))
            if l.kind == "mask":
                cur = g.node("Mask/Sigmoid", "Sigmoid", [y], T=_a_type(DT_FLOAT))
                continue
            if spec.norm == "batch":
                gm = _variable(g, l.name + "/norm/gamma", (l.cout,))
                bt = _variable(g, l.name + "/norm/beta", (l.cout,))
                mm = _variable(g, l.name + "/norm/moving_mean", (l.cout,))
                mv = _variable(g, l.name + "/norm/moving_variance", (l.cout,))
                y = g.node(l.name + "/norm/FusedBatchNorm", "FusedBatchNorm", [y, gm, bt, mm, mv],
                           T=_a_type(DT_FLOAT), epsilon=_a_f(1e-3), is_training=_a_b(False),
                           data_format=_a_s("NHWC"))
            elif spec.norm == "group":
                gm = _variable(g, l.name + "/norm/gamma", (l.cout,))
                bt = _variable(g, l.name + "/norm/beta", (l.cout,))
                y = g.node(l.name + "/norm/GroupNorm", "GroupNorm", [y, gm, bt], T=_a_type(DT_FLOAT),
                           groups=_a_i(spec.groups), epsilon=_a_f(1e-3))
            cur = g.node(l.name + "/Relu", "Relu", [y], T=_a_type(DT_FLOAT))
            outs[l.name] = cur
        elif l.kind == "pool":
            k = [1] + [2] * dims + [1]
            cur = g.node(l.name + "/" + pool_op, pool_op, [cur], T=_a_type(DT_FLOAT), ksize=_a_ints(k),
                         strides=_a_ints(k), padding=_a_s("VALID"),
                         data_format=_a_s("NDHWC" if dims == 3 else "NHWC"))
        elif l.kind == "tconv":
            k = _variable(g, l.name + "/kernel", l.kernel_shape(dims))
            b = _variable(g, l.name + "/bias", (l.cout,))
            shp = g.node(l.name + "/Shape", "Shape", [cur], T=_a_type(DT_FLOAT), out_type=_a_type(DT_INT32))
            s0 = g.const_i32(l.name + "/strided_slice/stack", [0], [1])
            s1 = g.const_i32(l.name + "/strided_slice/stack_1", [1], [1])
            s2 = g.const_i32(l.name + "/strided_slice/stack_2", [1], [1])
            bs = g.node(l.name + "/strided_slice", "StridedSlice", [shp, s0, s1, s2], T=_a_type(DT_INT32),
                        Index=_a_type(DT_INT32), shrink_axis_mask=_a_i(1), begin_mask=_a_i(0), end_mask=_a_i(0),
                        ellipsis_mask=_a_i(0), new_axis_mask=_a_i(0))
            side = img_size >> (l.level - 1)
            cs = [g.const_i32(l.name + "/stack/%d" % i, [v], []) for i, v in
                  enumerate([side] * dims + [l.cout])]
            st = g.node(l.name + "/stack", "Pack", [bs] + cs, T=_a_type(DT_INT32), N=_a_i(dims + 2), axis=_a_i(0))
            op = "Conv3DBackpropInputV2" if dims == 3 else "Conv2DBackpropInput"
            y = g.node(l.name + "/conv2d_transpose", op, [st, k, cur], T=_a_type(DT_FLOAT),
                       strides=_a_ints([1] + [2] * dims + [1]), padding=_a_s("SAME"),
                       data_format=_a_s("NDHWC" if dims == 3 else "NHWC"))
            cur = g.node(l.name + "/BiasAdd", "BiasAdd", [y, b], T=_a_type(DT_FLOAT), data_format=_a_s("NHWC"))
            pending_up = cur
        elif l.kind == "up":
            side = img_size >> (l.level - 1)
            if dims == 2:
                sz = g.const_i32(l.name + "/size", [side] * 2, [2])
                cur = g.node(l.name + "/ResizeNearestNeighbor", "ResizeNearestNeighbor", [cur, sz],
                             T=_a_type(DT_FLOAT), align_corners=_a_b(False))
            else:
                # [N, D, H, W, C] -> [N, D, 1, H, 1, W, 1, C] -> tile x2 on the unit axes
                # -> [N, 2D, 2H, 2W, C]: nearest-neighbour upsampling (UpSampling3D)
                lo, c = side // 2, l.cin
                s1 = g.const_i32(l.name + "/Reshape/shape", [-1, lo, 1, lo, 1, lo, 1, c], [8])
                r1 = g.node(l.name + "/Reshape", "Reshape", [cur, s1], T=_a_type(DT_FLOAT), Tshape=_a_type(DT_INT32))
                mu = g.const_i32(l.name + "/Tile/multiples", [1, 1, 2, 1, 2, 1, 2, 1], [8])
                t = g.node(l.name + "/Tile", "Tile", [r1, mu], T=_a_type(DT_FLOAT), Tmultiples=_a_type(DT_INT32))
                s2 = g.const_i32(l.name + "/Reshape_1/shape", [-1, side, side, side, c], [5])
                cur = g.node(l.name + "/Reshape_1", "Reshape", [t, s2], T=_a_type(DT_FLOAT),
                             Tshape=_a_type(DT_INT32))
            pending_up = cur
    if spec.norm == "batch":
        for l in spec.param_layers():
            if l.kind == "conv":
                variables += [(l.name + "/norm/moving_mean", (l.cout,)),
                              (l.name + "/norm/moving_variance", (l.cout,))]
    for n, shp in extra_vars:
        if n not in g.names:
            _variable(g, n, shp, DT_INT64 if n == "global_step" else DT_FLOAT)
        variables.append((n, tuple(shp)))
    _saver(g, [n for n, _ in variables])
    return g, variables


def _saver(g: _Graph, names: List[str]) -> None:
    """V2 Saver subgraph: SaveV2 / RestoreV2 over `names` (sorted, as tf.train.Saver)."""
    names = sorted(set(names))
    n = len(names)
    const = g.node("save/Const", "Const", dtype=_a_type(DT_STRING),
                   value=_a_tensor(_tensor_strings(["model"], [])))
    tn = g.node("save/SaveV2/tensor_names", "Const", dtype=_a_type(DT_STRING),
                value=_a_tensor(_tensor_strings(names, [n])))
    sl = g.node("save/SaveV2/shape_and_slices", "Const", dtype=_a_type(DT_STRING),
                value=_a_tensor(_tensor_strings([""] * n, [n])))
    dtypes = [DT_INT64 if x == "global_step" else DT_FLOAT for x in names]
    g.node("save/SaveV2", "SaveV2", [const, tn, sl] + names, dtypes=_a_types(dtypes))
    g.node("save/control_dependency", "Identity", [const, "^save/SaveV2"], T=_a_type(DT_STRING))
    rn = g.node("save/RestoreV2/tensor_names", "Const", dtype=_a_type(DT_STRING),
                value=_a_tensor(_tensor_strings(names, [n])))
    rs = g.node("save/RestoreV2/shape_and_slices", "Const", dtype=_a_type(DT_STRING),
                value=_a_tensor(_tensor_strings([""] * n, [n])))
    g.node("save/RestoreV2", "RestoreV2", [const, rn, rs], dtypes=_a_types(dtypes))
    assigns = []
    for i, v in enumerate(names):
        assigns.append(g.node("save/Assign_%d" % i if i else "save/Assign", "Assign", [v, "save/RestoreV2:%d" % i],
                              T=_a_type(dtypes[i]), validate_shape=_a_b(True), use_locking=_a_b(True)))
    g.node("save/restore_all", "NoOp", ["^" + a for a in assigns])


def _tensor_info(name: str, dims) -> bytes:
    # TensorInfo {name 1, dtype 2, tensor_shape 3}
    return _s(1, name) + _fv(2, DT_FLOAT) + _fbytes(3, _shape(dims))


def _saver_def() -> bytes:
    # SaverDef: filename_tensor_name 1, save_tensor_name 2, restore_op_name 3, max_to_keep 4,
    # sharded 5, keep_checkpoint_every_n_hours 6 (float), version 7 (V2 = 2)
    import struct
    return (_s(1, "save/Const:0") + _s(2, "save/control_dependency:0") + _s(3, "save/restore_all")
            + _fv(4, 5) + _fv(5, 0) + _field(6, 5, struct.pack("<f", 10000.0)) + _fv(7, 2))


def _variable_def(name: str) -> bytes:
    # VariableDef: variable_name 1, initializer_name 2, snapshot_name 3
    return _s(1, name + ":0") + _s(2, name + "/Assign") + _s(3, name + "/read:0")


def meta_graph_def(spec, img_size: int, tags: Sequence[str] = (), signature: bool = False,
                   extra_vars: Sequence[Tuple[str, Tuple[int, ...]]] = ()) -> bytes:
    """MetaGraphDef {meta_info_def 1, graph_def 2, saver_def 3, collection_def 4,
    signature_def 5}."""
    g, variables = build_graph(spec, img_size, extra_vars)
    info = _s(1, "") + b"".join(_s(4, t) for t in tags) + _s(5, TF_VERSION) + _s(6, "unknown")
    trainable = [n for n, _ in spec.variables()]
    coll = b""
    for cname, names in (("trainable_variables", trainable), ("variables", [n for n, _ in variables])):
        bl = b"".join(_fbytes(1, _variable_def(n)) for n in names)
        coll += _fbytes(4, _map_entry(cname, _fbytes(2, bl)))          # CollectionDef.bytes_list
    body = _fbytes(1, info) + _fbytes(2, g.encode()) + _fbytes(3, _saver_def()) + coll
    if signature:
        img = [-1] + [img_size] * spec.dims
        sig = (_fbytes(1, _map_entry("image", _tensor_info("Placeholder:0", img + [spec.in_channels])))
               + _fbytes(2, _map_entry("prediction", _tensor_info("Mask/Sigmoid:0", img + [spec.n_cl_out])))
               + _s(3, "tensorflow/serving/predict"))
        body += _fbytes(5, _map_entry("intel_unet_brats_model", sig))
    return body


def write_saved_model(directory: str, spec, img_size: int) -> str:
    """saved_model.pb = SavedModel {saved_model_schema_version 1, meta_graphs 2} with one
    MetaGraphDef tagged 'serve' carrying the intel_unet_brats_model signature."""
    mg = meta_graph_def(spec, img_size, tags=["serve"], signature=True)
    path = os.path.join(directory, "saved_model.pb")
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(_fv(1, 1) + _fbytes(2, mg))
    os.replace(tmp, path)
    return path


def write_meta(prefix: str, spec, img_size: int, var_shapes: Sequence[Tuple[str, Tuple[int, ...]]]) -> str:
    """<prefix>.meta: the Saver's MetaGraphDef (graph over every checkpointed variable:
    weights, Adam slots, beta powers, global_step)."""
    mg = meta_graph_def(spec, img_size, extra_vars=var_shapes)
    path = prefix + ".meta"
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(mg)
    os.replace(tmp, path)
    return path


# ------------------------------------------------------------------ reading it back
def _i64(v: int) -> int:
    return v - (1 << 64) if v >= (1 << 63) else v


def _parse_shape(b: bytes) -> List[int]:
    from .tf_bundle import _parse
    return [_i64(_parse(d).get(1, [0])[0]) for d in _parse(b).get(2, [])]


def graph_nodes(graph_def: bytes) -> Dict[str, dict]:
    """GraphDef bytes -> {name: {"op", "inputs", "attr": {key: AttrValue fields}}}."""
    from .tf_bundle import _parse
    out = {}
    for nb in _parse(graph_def).get(1, []):
        n = _parse(nb)
        attrs = {}
        for e in n.get(5, []):
            kv = _parse(e)
            attrs[kv[1][0].decode()] = _parse(kv[2][0]) if 2 in kv else {}
        out[n[1][0].decode()] = {"op": n[2][0].decode(), "inputs": [i.decode() for i in n.get(3, [])],
                                 "attr": attrs}
    return out


def read_saved_model(path: str) -> dict:
    """saved_model.pb -> {"tags", "signatures": {name: {"inputs": {k: tensor}, "outputs":
    {k: tensor}, "method"}}, "nodes", "variables": {name: shape}} of its first MetaGraph."""
    from .tf_bundle import _parse
    sm = _parse(open(path, "rb").read())
    mg = _parse(sm[2][0])
    info = _parse(mg[1][0])
    sigs = {}
    for e in mg.get(5, []):
        kv = _parse(e)
        sd = _parse(kv[2][0])
        io = []
        for f in (1, 2):
            m = {}
            for te in sd.get(f, []):
                tkv = _parse(te)
                ti = _parse(tkv[2][0])
                m[tkv[1][0].decode()] = {"name": ti[1][0].decode(), "shape": _parse_shape(ti[3][0]) if 3 in ti else None}
            io.append(m)
        sigs[kv[1][0].decode()] = {"inputs": io[0], "outputs": io[1],
                                   "method": sd[3][0].decode() if 3 in sd else ""}
    nodes = graph_nodes(mg[2][0])
    var_shapes = {k: _parse_shape(v["attr"]["shape"][7][0]) for k, v in nodes.items() if v["op"] == "VariableV2"}
    return {"tags": [t.decode() for t in info.get(4, [])], "signatures": sigs, "nodes": nodes,
            "variables": var_shapes, "meta_graph": mg}


def spec_from_graph(sm: dict, signature: str = "intel_unet_brats_model"):
    """(UNetSpec, img_size) of an exported inference graph: input channels / rank / size
    from the signature's input placeholder, the base width from conv1a's kernel, the
    depth from the max-pool count, the decoder variant from the transposed-conv /
    upsampling nodes, the normalisation from FusedBatchNorm / GroupNorm nodes, the
    classes from the Mask kernel.  (Dropout is not part of an inference graph: the
    spec keeps the default rate, which only training uses.)"""
    from ..models.spec import UNetSpec
    nodes, var = sm["nodes"], sm["variables"]
    sig = sm["signatures"].get(signature) or next(iter(sm["signatures"].values()))
    inp = next(iter(sig["inputs"].values()))["name"].split(":")[0]
    out = next(iter(sig["outputs"].values()))["name"].split(":")[0]
    if inp not in nodes or out not in nodes:
        raise ValueError("signature tensors %s / %s are not in the graph" % (inp, out))
    shp = _parse_shape(nodes[inp]["attr"]["shape"][7][0])
    dims = len(shp) - 2
    ops = [v["op"] for v in nodes.values()]
    depth = sum(1 for o in ops if o in ("MaxPool", "MaxPool3D"))
    gn = [v for v in nodes.values() if v["op"] == "GroupNorm"]
    norm = "batch" if "FusedBatchNorm" in ops else ("group" if gn else "none")
    groups = _i64(gn[0]["attr"]["groups"][3][0]) if gn else 8
    ups = any(k.startswith("up") for k, v in nodes.items() if v["op"] in ("ResizeNearestNeighbor", "Tile"))
    spec = UNetSpec(in_channels=shp[-1], n_cl_out=var["Mask/kernel"][-1], base=var["conv1a/kernel"][-1],
                    depth=depth, use_upsampling=ups, dims=dims, norm=norm, groups=groups)
    for name, s in spec.variables():
        if tuple(var.get(name, ())) != tuple(s):
            raise ValueError("graph variable %s has shape %s, the recovered spec expects %s"
                             % (name, var.get(name), s))
    return spec, shp[1]
