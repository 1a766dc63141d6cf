"""Extract the input assets the integrator needs from the reference checkout (run once,
in the build container; the outputs are committed under hikari_amd/assets/).

* src/noise/LDR_RGBA_{0..15}.png -> blue_noise_16x64x64_rgba8.bin (raw RGBA8, texture-major).
  The reference loads them with `Image::from_buffer(.., is_srgb=false)` (lib.rs:189-219),
  i.e. as linear Rgba8Unorm, so the bytes are used as-is.
* assets/models/cornell.glb is copied verbatim (input data for examples/cornell.rs).
* assets/models/City/scene.gltf -> city_layout.json: node transforms, per-mesh POSITION
  bounds, vertex/index counts and material emissive factors (the geometry itself,
  scene.bin, is missing from the checkout; .MISSING_LARGE_BLOBS:1).
"""
import json
import shutil
import sys
from pathlib import Path

import numpy as np

REF = Path(sys.argv[1] if len(sys.argv) > 1 and __name__ == "__main__" else "/root/reference")
OUT = Path(__file__).resolve().parent.parent / "hikari_amd" / "assets"


def blue_noise(ref: Path) -> np.ndarray:
    """The 16 noise textures decoded: (16, 64, 64, 4) uint8, texture-major."""
    from PIL import Image
    tex = []
    for i in range(16):
        im = Image.open(ref / "src" / "noise" / f"LDR_RGBA_{i}.png")
        a = np.asarray(im.convert("RGBA"), dtype=np.uint8)
        assert a.shape == (64, 64, 4), a.shape
        tex.append(a)
    return np.stack(tex)


def city_layout(ref: Path) -> dict:
    """The City proxy's layout from assets/models/City/scene.gltf."""
    g = json.loads((ref / "assets" / "models" / "City" / "scene.gltf").read_text())
    layout = {"source": "assets/models/City/scene.gltf (JSON only; scene.bin missing)",
              "scene_roots": g["scenes"][g.get("scene", 0)]["nodes"], "nodes": [], "meshes": [], "materials": []}
    for n in g["nodes"]:
        layout["nodes"].append({k: n[k] for k in ("mesh", "children", "translation", "rotation", "scale", "matrix")
                                if k in n})
    for m in g["meshes"]:
        prims = []
        for p in m["primitives"]:
            pos = g["accessors"][p["attributes"]["POSITION"]]
            prims.append({
                "min": pos["min"], "max": pos["max"], "vertex_count": pos["count"],
                "index_count": g["accessors"][p["indices"]]["count"] if "indices" in p else pos["count"],
                "has_normal": "NORMAL" in p["attributes"], "has_uv": "TEXCOORD_0" in p["attributes"],
                "material": p.get("material"), "mode": p.get("mode", 4)})
        layout["meshes"].append(prims)
    for mat in g["materials"]:
        pbr = mat.get("pbrMetallicRoughness", {})
        layout["materials"].append({
            "name": mat.get("name"), "base_color": pbr.get("baseColorFactor", [1, 1, 1, 1]),
            "metallic": pbr.get("metallicFactor", 1.0), "roughness": pbr.get("roughnessFactor", 1.0),
            "emissive": mat.get("emissiveFactor", [0, 0, 0])})
    return layout


def city_layout_text(layout: dict) -> str:
    return json.dumps(layout, separators=(",", ":"))


def main():
    OUT.mkdir(parents=True, exist_ok=True)
    blue_noise(REF).tofile(OUT / "blue_noise_16x64x64_rgba8.bin")
    shutil.copyfile(REF / "assets" / "models" / "cornell.glb", OUT / "cornell.glb")
    (OUT / "city_layout.json").write_text(city_layout_text(city_layout(REF)))


if __name__ == "__main__":
    main()
