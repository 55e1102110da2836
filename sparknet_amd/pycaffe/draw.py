"""Net graph drawing (caffe/python/caffe/draw.py).  pydot is not available here, so the
graph is produced as Graphviz DOT text — layers as boxes (coloured by type, labelled
with kernel / stride / pad), blobs as octagons, edges labelled with blob names — and
rendered to an image only when a ``dot`` executable is on PATH."""
from __future__ import annotations

import shutil
import subprocess

from .. import proto

_COLORS = {"Convolution": "#FF5050", "Deconvolution": "#FF5050", "Pooling": "#FF9900",
           "InnerProduct": "#CC33FF", "LRN": "#66CCFF"}
_BLOB_COLOR = "#E0E0E0"


def _pool_name(v: int) -> str:
    return {0: "MAX", 1: "AVE", 2: "STOCHASTIC"}.get(int(v), str(v))


def layer_label(layer, rankdir: str = "LR") -> str:
    sep = "\\n" if rankdir in ("TB", "BT") else " "
    t = layer.type
    if t in ("Convolution", "Deconvolution"):
        p = layer.convolution_param
        k = list(p.kernel_size) or [p.kernel_h]
        s = list(p.stride) or [p.stride_h or 1]
        pad = list(p.pad) or [p.pad_h]
        return f"{layer.name}{sep}({t}){sep}kernel size: {k[0]}{sep}stride: {s[0]}{sep}pad: {pad[0]}"
    if t == "Pooling":
        p = layer.pooling_param
        return (f"{layer.name}{sep}({_pool_name(p.pool)} {t}){sep}kernel size: {p.kernel_size}{sep}"
                f"stride: {p.stride}{sep}pad: {p.pad}")
    return f"{layer.name}{sep}({t})"


def get_graph_dot(net_param, rankdir: str = "LR", label_edges: bool = True) -> str:
    """DOT source of a NetParameter's layer/blob graph."""
    lines = [f'digraph "{net_param.name or "net"}" {{', f"  rankdir={rankdir};"]
    blobs = set()
    for i, layer in enumerate(net_param.layer):
        lid = f"layer_{i}"
        color = _COLORS.get(layer.type, "#6495ED")
        lines.append(f'  {lid} [shape=record, style=filled, fillcolor="{color}", '
                     f'label="{layer_label(layer, rankdir)}"];')
        for b in layer.bottom:
            blobs.add(b)
            lab = f' [label="{b}"]' if label_edges else ""
            lines.append(f'  "blob_{b}" -> {lid}{lab};')
        for t in layer.top:
            blobs.add(t)
            lines.append(f'  {lid} -> "blob_{t}";')
    for b in sorted(blobs):
        lines.append(f'  "blob_{b}" [shape=octagon, style=filled, fillcolor="{_BLOB_COLOR}", label="{b}"];')
    lines.append("}")
    return "\n".join(lines) + "\n"


def draw_net(net_param, rankdir: str = "LR", ext: str = "png") -> bytes:
    """Rendered image bytes (needs Graphviz ``dot``) or, for ext == 'dot', the DOT text."""
    dot = get_graph_dot(net_param, rankdir)
    if ext == "dot":
        return dot.encode()
    exe = shutil.which("dot")
    if exe is None:
        raise RuntimeError("Graphviz 'dot' is not installed; use ext='dot' for the DOT source")
    return subprocess.run([exe, f"-T{ext}"], input=dot.encode(), capture_output=True, check=True).stdout


def draw_net_to_file(net_param, filename: str, rankdir: str = "LR") -> None:
    if isinstance(net_param, str):
        net_param = proto.read_net(net_param)
    ext = filename.rsplit(".", 1)[-1] if "." in filename else "dot"
    with open(filename, "wb") as f:
        f.write(draw_net(net_param, rankdir, ext))
