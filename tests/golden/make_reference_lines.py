"""Writes tests/golden/reference_lines.json: the line count of each reference
source file the repo cites (file:line), and the line of each declaration the
boundary header maps (Renderer.h methods, Primitive.h types, ...).  Numbers
only -- no reference text is stored.  Run in a container that has
/root/reference:

    python tests/golden/make_reference_lines.py
"""
import json
import os
import re

REF = "/root/reference/PathTracerAP"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_lines.json")
FILES = ["Renderer.cpp", "Renderer.h", "Scene.cpp", "Scene.h", "Primitive.h", "utility.h", "Config.h",
         "GPUMemoryPool.h", "main.cpp", "Experimentation.h"]
# symbol -> regex matched against a line (first non-comment match wins)
SYMBOLS = {
    "Renderer.h": {"class Renderer": r"^class Renderer\b", "allocateOnGPU": r"\ballocateOnGPU\(",
                   "renderLoop": r"\brenderLoop\(", "renderImage": r"\brenderImage\(", "free": r"\bfree\(\);"},
    "Primitive.h": {"IndexRange": r"struct IndexRange\b", "Vertex": r"struct Vertex\b", "Triangle": r"struct Triangle\b",
                    "BoundingBox": r"struct BoundingBox\b", "Material": r"struct Material\b",
                    "MaterialType": r"enum MaterialType\b", "Mesh": r"struct Mesh\b", "Model": r"struct Model\b",
                    "EntityType": r"enum EntityType\b", "Voxel": r"struct Voxel\s*$", "Grid": r"struct Grid\b"},
    "Scene.h": {"class Scene": r"^class Scene\b", "Scene(string config)": r"\bScene\(string config\)"},
    "Scene.cpp": {"Scene::Scene": r"^Scene::Scene\(", "Scene::loadAndProcessMeshFile": r"Scene::loadAndProcessMeshFile\(",
                  "Scene::processMesh": r"Scene::processMesh\(", "computeVoxelIndex": r"^void computeVoxelIndex\(",
                  "Scene::addMeshesToGrid": r"Scene::addMeshesToGrid\("},
    "Renderer.cpp": {"Renderer::renderImage": r"Renderer::renderImage\(", "Renderer::allocateOnGPU": r"Renderer::allocateOnGPU\(",
                     "Renderer::free": r"Renderer::free\(", "Renderer::renderLoop": r"Renderer::renderLoop\(",
                     "computeRayGridIntersection": r"^bool computeRayGridIntersection\(",
                     "computeRaySceneIntersectionKernel": r"^void computeRaySceneIntersectionKernel\(",
                     "shadeRayKernel": r"^void shadeRayKernel\(", "generateRaysKernel": r"^void generateRaysKernel\("},
}


def scan(ref=REF):
    out = {"source": "line counts (str.splitlines) of purvakulkarni15/PathTracerAP/PathTracerAP/<file> and the "
                     "line of each named declaration; tests/golden/make_reference_lines.py", "files": {}}
    for f in FILES:
        with open(os.path.join(ref, f), encoding="utf-8", errors="replace") as fh:
            lines = fh.read().splitlines()
        d = {"lines": len(lines)}
        if f in SYMBOLS:
            d["symbols"] = {}
            for name, rx in SYMBOLS[f].items():
                r = re.compile(rx)
                hits = [i + 1 for i, l in enumerate(lines) if r.search(l) and not l.strip().startswith("//")]
                d["symbols"][name] = hits[0]
        out["files"][f] = d
    return out


if __name__ == "__main__":
    with open(OUT, "w") as fh:
        json.dump(scan(), fh, indent=1)
        fh.write("\n")
    print("wrote", OUT)
