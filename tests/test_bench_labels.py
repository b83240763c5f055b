"""bench.py's workload labels follow SURVEY.md 8(d)'s config names (host logic, no GPU)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def test_config_ids():
    assert bench._config_id("S0", 256, 256, 64, 1) == "C1"
    assert bench._config_id("T", 1920, 1080, 128, 1) == "C2"
    assert bench._config_id("T", 4096, 4096, 256, 1) == "C3"
    assert bench._config_id("T", 4096, 4096, 256, 8) == "C4"
    assert bench._config_id("O", 8192, 8192, 512, 1) == "C5"
    assert bench._config_id("O", 4096, 4096, 256, 1) == "custom"
