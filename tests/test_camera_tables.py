"""The host camera tables (rtx/scene.py camera_tables) against the reference's loop forms
(provided/scene.py:36-61, :118-138): the running sums x += dx / y += dy and the sunflower
spread, evaluated step by step with numpy fp64 scalars as the reference does. The product
computes them vectorised (add.accumulate, cached trig terms); the values must be the same
bits."""
import numpy as np
import pytest

from rtx.helperclasses import sunflower, sunflower_many
from rtx.scene import running_sum


def loop_running_sum(x0, dx, n):
    out = np.empty(n, np.float64)
    x = x0
    for i in range(n):
        out[i] = x
        x += dx
    return out


def loop_sunflower(num_points, origin, radius):
    phi = (1 + np.sqrt(5)) / 2
    angle_stride = 2 * np.pi / phi
    out = np.zeros((num_points, 3), dtype=np.float32)
    ox, oy, oz = float(origin[0]), float(origin[1]), origin[2]
    for k in range(1, num_points + 1):
        r = radius * np.sqrt(k - 0.5) / np.sqrt(num_points - 0.5)
        theta = k * angle_stride
        out[k - 1] = np.array([r * np.cos(theta) + ox, r * np.sin(theta) + oy, oz], dtype=np.float64).astype(np.float32)
    return out


@pytest.mark.parametrize("seed", range(20))
def test_running_sum_is_the_loop(seed):
    rng = np.random.RandomState(seed)
    n = int(rng.randint(1, 5000))
    x0 = np.float64(rng.uniform(-3, 3)) + (0.5 + np.int64(rng.randint(0, 4000))) * np.float64(rng.uniform(1e-4, 1e-2))
    dx = np.float64(rng.uniform(1e-5, 1e-2))
    assert running_sum(x0, dx, n).tobytes() == loop_running_sum(x0, dx, n).tobytes()


@pytest.mark.parametrize("n", [1, 2, 3, 4, 7, 15, 16, 32, 33, 64, 100])
def test_sunflower_is_the_loop(n):
    rng = np.random.RandomState(n)
    for _ in range(5):
        origin = rng.uniform(-10, 10, 3).astype(np.float32)
        radius = float(rng.uniform(0, 2))
        assert sunflower(n, origin, radius).tobytes() == loop_sunflower(n, origin, radius).tobytes()
    origins = rng.uniform(-10, 10, (9, 3)).astype(np.float32)
    many = sunflower_many(n, origins, 0.37)
    for k in range(len(origins)):
        assert many[k].tobytes() == loop_sunflower(n, origins[k], 0.37).tobytes()
