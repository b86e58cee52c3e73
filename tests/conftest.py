import os
import sys

# The tests pin which kernel renders: scene-specialized kernels compile before the render
# that needs them returns (the product default, option jit_async 1, renders with the
# generic kernel meanwhile; tests/test_gpu_jit_cache.py covers that path). Read by the
# library once, at its first option lookup.
os.environ.setdefault("RTX_JIT_ASYNC", "0")
# The suite builds hundreds of scenes, each with kernels specialized on its records or CSG
# trees; the product keeps 8 idle modules loaded and 64 code objects on disk, so the same
# scene's kernels (NovelScene1's CSG passes: ~20 s of hiprtc) would compile again in later
# tests. Keep them all for the session (what is cached, not what renders).
os.environ.setdefault("RTX_JIT_IDLE_BAKED", "1024")
os.environ.setdefault("RTX_JIT_DISK_BAKED", "100000")

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (REPO, os.path.join(REPO, "python-raytracer_amd"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librtx.so)")
