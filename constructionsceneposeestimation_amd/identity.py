"""Instance identity: prim path -> (object root, class name, class id).

Restates the semantics of the reference's ``get_object_root``
(generate_construction_data.py:144-233), its class table
``construction_class`` (:69-106), ``CRANE_PART_CHILD_MAP`` (:110-121) and
the crane-part map built by ``build_crane_part_map`` (:1234-1279).  These
decide which integer id the GPU instance-fill writes for every pixel: every
mesh that resolves to the same object root shares that root's ``inst_idx``;
unmatched meshes (e.g. the ground) write -1 (background, :1909-1910).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Tuple

CONSTRUCTION_CLASS: Dict[str, int] = {
    "trafficcone": 0, "cone": 0,
    "tree": 1,
    "fence": 2, "fencing": 2, "construction_site": 2,
    "crane": 3, "pk7": 3,
    "cranebase": 6, "cranecolumn": 7, "craneboom": 8, "cranetelescopic": 9,
    "dumper": 4, "09684481": 4,
    "human": 5, "dhgen": 5, "skelroot": 5,
}

CRANE_PART_CHILD_MAP: Dict[str, Tuple[str, int]] = {
    "s104gg03a_sw": ("cranebase", 6),
    "s104s01kb_sw": ("cranebase", 6),
    "s104hz01ka_sw": ("cranecolumn", 7),
    "s104h01kb_sw": ("cranecolumn", 7),
    "s104hz02ka_sw": ("cranecolumn", 7),
    "s104kz01ka_sw": ("cranecolumn", 7),
    "tn__s104ekb_as_sw_jj7": ("craneboom", 8),
    "s104kz02ka_sw": ("cranetelescopic", 9),
    "tn__hhk320ka_sw_lg": ("cranetelescopic", 9),
    "tn__hhk319_sw_od": ("cranetelescopic", 9),
}

CRANE_ROOT = "/World/GroundPlane/tn__Pk7501SLD_PNR3879_fPM"
DUMPER_ROOT = "/World/GroundPlane/tn__09684481_"
HUMAN_ROOT = "/World/GroundPlane/DHGen"

_BASE_KW = ("base", "chassis", "footer", "support", "grund", "fahrwerk")
_COLUMN_KW = ("column", "turret", "mast", "tower", "saeule", "drehwerk", "oberwagen")
_BOOM_KW = ("boom", "arm", "jib", "ausleger")
_TELE_KW = ("telescop", "extension", "teleskop", "auszug")

Root = Tuple[Optional[str], Optional[str], Optional[int]]


def build_crane_part_map(crane_descendants: Iterable[Tuple[str, str]]) -> Dict[str, Tuple[str, int]]:
    """Map every prim under the crane root to its part class.

    ``crane_descendants`` yields ``(first_level_child_path, descendant_path)``
    pairs (the child itself included), as ``Usd.PrimRange`` would
    (generate_construction_data.py:1254-1268).  Unknown first-level children
    map to the whole crane ("crane", 3).
    """
    out: Dict[str, Tuple[str, int]] = {}
    for child, desc in crane_descendants:
        name = child.rstrip("/").split("/")[-1].lower()
        out[desc] = CRANE_PART_CHILD_MAP.get(name, ("crane", 3))
    return out


def get_object_root(prim_path: str, crane_part_map: Optional[Dict[str, Tuple[str, int]]] = None) -> Root:
    """(object_root, class_name, class_id) or (None, None, None).

    Same decision order as generate_construction_data.py:151-233: fence,
    tree, cone, crane (part map, first-level child, keywords, whole crane),
    dumper, human, then the first ``construction_class`` key contained in
    the lower-cased path (dict order), else unmatched.
    """
    low = prim_path.lower()
    if "fencing_height_" in low:
        parts = prim_path.split("/")
        for i, part in enumerate(parts):
            if "Fencing_height_" in part:
                return "/".join(parts[:i + 1]), "fence", CONSTRUCTION_CLASS["fence"]
    if "/world/tree/tree" in low:
        parts = prim_path.split("/")
        if len(parts) >= 4:
            return "/".join(parts[:4]), "tree", CONSTRUCTION_CLASS["tree"]
    if "/cone001" in low:
        parts = prim_path.split("/")
        for i, part in enumerate(parts):
            if part.lower().startswith("cone001"):
                return "/".join(parts[:i + 1]), "trafficcone", CONSTRUCTION_CLASS["trafficcone"]
    if "pk7501sld" in low or "pk7" in low:
        if crane_part_map and prim_path in crane_part_map:
            name, cid = crane_part_map[prim_path]
            return CRANE_ROOT + "#" + name, name, cid
        if prim_path.startswith(CRANE_ROOT + "/") or low.startswith(CRANE_ROOT.lower() + "/"):
            first = prim_path[len(CRANE_ROOT) + 1:].split("/")[0].lower()
            if first in CRANE_PART_CHILD_MAP:
                name, cid = CRANE_PART_CHILD_MAP[first]
                return CRANE_ROOT + "#" + name, name, cid
        sub = low[low.find("pk7"):]
        for kws, name in ((_BASE_KW, "cranebase"), (_COLUMN_KW, "cranecolumn"),
                          (_BOOM_KW, "craneboom"), (_TELE_KW, "cranetelescopic")):
            if any(k in sub for k in kws):
                return CRANE_ROOT + "#" + name, name, CONSTRUCTION_CLASS[name]
        return CRANE_ROOT, "crane", CONSTRUCTION_CLASS["crane"]
    if "09684481" in low:
        return DUMPER_ROOT, "dumper", CONSTRUCTION_CLASS["dumper"]
    if "dhgen" in low:
        return HUMAN_ROOT, "human", CONSTRUCTION_CLASS["human"]
    for key, cid in CONSTRUCTION_CLASS.items():
        if key in low:
            return prim_path, key, cid
    return None, None, None


def assign_instances(mesh_paths: List[str], crane_part_map=None) -> Tuple[List[int], List[dict]]:
    """Aggregate mesh paths into object roots in first-appearance order
    (generate_construction_data.py:1857-1891).

    Returns ``(inst_of_mesh, objects)``: ``inst_of_mesh[i]`` is the
    ``inst_idx`` of ``mesh_paths[i]`` (-1 = unmatched/background) and
    ``objects[k]`` = ``{inst_idx, class_id, class_name, prim_path, mesh_paths}``.
    The reference iterates Replicator's bbox primPaths; this build iterates
    the scene-traversal order, which makes ``inst_idx`` stable per scene.
    """
    roots: Dict[str, dict] = {}
    inst_of_mesh: List[int] = []
    for p in mesh_paths:
        root, name, cid = get_object_root(p, crane_part_map)
        if root is None:
            inst_of_mesh.append(-1)
            continue
        if root not in roots:
            roots[root] = {"inst_idx": len(roots), "class_id": cid, "class_name": name,
                           "prim_path": root, "mesh_paths": []}
        roots[root]["mesh_paths"].append(p)
        inst_of_mesh.append(roots[root]["inst_idx"])
    return inst_of_mesh, list(roots.values())
