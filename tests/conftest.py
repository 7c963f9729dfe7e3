import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)

ASSETS = os.path.join(ROOT, "assets")
CORNELL_OBJ = os.path.join(ASSETS, "CornellBox", "CornellBox-Empty-CO.obj")
CORNELL_MTL = os.path.join(ASSETS, "CornellBox", "CornellBox-Empty-CO.mtl")
CUBE_OBJ = os.path.join(ASSETS, "shapes", "cube.obj")
SPHERE_OBJ = os.path.join(ASSETS, "shapes", "sphere.obj")
CUBE_KD = "*Kd 0.9041462985304743 0.5854651848798454 0.007022117649276849*"  # scenes/0.txt

# object records (pos, ori, scl, obj, mtl) -- the oracle's and the product's input
CORNELL = [((0, 0, 4), (0, 0, 0), (2, 2, 2), CORNELL_OBJ, CORNELL_MTL)]
SCENE0 = CORNELL + [((0, -1.5, 4), (0, 0, 0), (1, 1, 1), CUBE_OBJ, CUBE_KD)]
# BASELINE.json configs[2] as the north_star names it: "CornellBox + shapes/sphere.obj + cube.obj" --
# scenes/0.txt plus a sphere (assets/northstar.txt; no shipped scene file uses sphere.obj), 1310 triangles
NORTHSTAR = SCENE0 + [((-1.2, -1.35, 4.6), (0, 0, 0), (1.2, 1.2, 1.2), SPHERE_OBJ, "*Kd 0.2 0.6 0.3*")]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long CPU test")


def product_scene(records, device=True):
    from inverse_path_tracer_amd.scene import ObjectSpec, Scene

    return Scene([ObjectSpec(r[3], r[4], r[0], r[1], r[2]) for r in records], device=device)


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib

    oracle_lib.build()
    return oracle_lib
