"""Writers for small synthetic mesh files (PLY ascii / binary, binary FBX 7.x)
used by the loader tests.  The reference ships no mesh the image can decode
with the reference's own loader (its assimp binaries are Win32 only), so the
loaders are checked on files built here from known polygons: parity of the
loaders themselves is "unpinned" against the reference."""
from __future__ import annotations

import struct
import zlib

import numpy as np

# ----------------------------------------------------------------------- PLY


def write_ply(path, verts, faces, normals=None, uvs=None, fmt="ascii"):
    """verts (n,3), faces list of index lists, optional normals (n,3), uvs (n,2)."""
    verts = np.asarray(verts, np.float32)
    head = ["ply", f"format {fmt} 1.0", "comment srr test mesh", f"element vertex {len(verts)}",
            "property float x", "property float y", "property float z"]
    if normals is not None:
        head += ["property float nx", "property float ny", "property float nz"]
    if uvs is not None:
        head += ["property float s", "property float t"]
    head += [f"element face {len(faces)}", "property list uchar int vertex_indices", "end_header"]
    cols = [verts]
    if normals is not None:
        cols.append(np.asarray(normals, np.float32))
    if uvs is not None:
        cols.append(np.asarray(uvs, np.float32))
    vt = np.concatenate(cols, axis=1)
    with open(path, "wb") as f:
        f.write(("\n".join(head) + "\n").encode())
        if fmt == "ascii":
            for row in vt:
                f.write((" ".join(repr(float(x)) for x in row) + "\n").encode())
            for fc in faces:
                f.write((" ".join(str(x) for x in [len(fc), *fc]) + "\n").encode())
        else:
            e = "<" if fmt == "binary_little_endian" else ">"
            for row in vt:
                f.write(struct.pack(e + "f" * len(row), *row.tolist()))
            for fc in faces:
                f.write(struct.pack(e + "B" + "i" * len(fc), len(fc), *fc))


# ----------------------------------------------------------------------- FBX


class Node:
    def __init__(self, name, props=(), kids=()):
        self.name, self.props, self.kids = name, list(props), list(kids)


def _prop(p, compress):
    kind, v = p
    if kind == "S":
        b = v.encode()
        return b"S" + struct.pack("<I", len(b)) + b
    if kind in "ILDY":
        return kind.encode() + struct.pack({"I": "<i", "L": "<q", "D": "<d", "Y": "<h"}[kind], v)
    # arrays: d (double), i (int32), l (int64)
    fmt = {"d": "<d", "i": "<i", "l": "<q", "f": "<f"}[kind]
    raw = b"".join(struct.pack(fmt, x) for x in v)
    if compress:
        z = zlib.compress(raw)
        return kind.encode() + struct.pack("<III", len(v), 1, len(z)) + z
    return kind.encode() + struct.pack("<III", len(v), 0, len(raw)) + raw


def _node(n, off, wide, compress):
    pb = b"".join(_prop(p, compress) for p in n.props)
    name = n.name.encode()
    hdr = 25 if wide else 13
    body_off = off + hdr + len(name) + len(pb)
    kids = b""
    for k in n.kids:
        kids += _node(k, body_off + len(kids), wide, compress)
    if n.kids:
        kids += b"\0" * hdr
    end = body_off + len(kids)
    f = "<QQQ" if wide else "<III"
    return struct.pack(f, end, len(n.props), len(pb)) + bytes([len(name)]) + name + pb + kids


def write_fbx(path, top_nodes, version=7400, compress=False):
    wide = version >= 7500
    out = b"Kaydara FBX Binary  \0\x1a\0" + struct.pack("<I", version)
    for n in top_nodes:
        out += _node(n, len(out), wide, compress)
    out += b"\0" * (25 if wide else 13)
    with open(path, "wb") as f:
        f.write(out)


def fbx_geometry(gid, verts, polys, normals_pv=None, uv=None, uv_index=None, materials=None):
    """A Geometry node: polys are vertex-index lists; normals_pv per polygon
    vertex (Direct); uv data + per-polygon-vertex UVIndex (IndexToDirect);
    materials per polygon (ByPolygon)."""
    pvi = []
    for p in polys:
        pvi += list(p[:-1]) + [-p[-1] - 1]
    kids = [Node("Vertices", [("d", [float(x) for x in np.ravel(verts)])]),
            Node("PolygonVertexIndex", [("i", pvi)])]
    if normals_pv is not None:
        kids.append(Node("LayerElementNormal", [("I", 0)], [
            Node("MappingInformationType", [("S", "ByPolygonVertex")]),
            Node("ReferenceInformationType", [("S", "Direct")]),
            Node("Normals", [("d", [float(x) for x in np.ravel(normals_pv)])])]))
    if uv is not None:
        kids.append(Node("LayerElementUV", [("I", 0)], [
            Node("MappingInformationType", [("S", "ByPolygonVertex")]),
            Node("ReferenceInformationType", [("S", "IndexToDirect")]),
            Node("UV", [("d", [float(x) for x in np.ravel(uv)])]),
            Node("UVIndex", [("i", list(uv_index))])]))
    if materials is not None:
        kids.append(Node("LayerElementMaterial", [("I", 0)], [
            Node("MappingInformationType", [("S", "ByPolygon")]),
            Node("ReferenceInformationType", [("S", "IndexToDirect")]),
            Node("Materials", [("i", list(materials))])]))
    return Node("Geometry", [("L", gid), ("S", "Geometry::mesh\0\x01Geometry"), ("S", "Mesh")], kids)


def fbx_model(mid, name):
    return Node("Model", [("L", mid), ("S", f"Model::{name}\0\x01Model"), ("S", "Mesh")])


def fbx_scene(objects, connections):
    """connections: (child, parent) object-object links, 0 = scene root."""
    return [Node("FBXHeaderExtension", [], [Node("FBXVersion", [("I", 7400)])]),
            Node("Objects", [], objects),
            Node("Connections", [], [Node("C", [("S", "OO"), ("L", c), ("L", p)]) for c, p in connections])]
