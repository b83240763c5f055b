"""raymarching_amd -- MI355X-native SDF sphere-tracing pass (HIP, gfx950).

Drop-in for the full-screen ray-march fragment pass of cahekp/Raymarching
(common.frag + output_shader.frag / template.frag).  The compute lives in
``librm.so`` (hand-written HIP kernels behind the C ABI of include/rm.h);
this package is the host-side mirror of the reference's
ShaderLoader / sf::Shader / RenderTexture surface plus the row-sharded
multi-GPU frame (``frame.py``).
"""
from ._lib import EXPORTS, LIB_PATH, RmError, lib  # noqa: F401
from .api import (Comm, Renderer, RenderTexture, Shader, ShaderLoader, comm_get_id, compile_scene,  # noqa: F401
                  cycle_rows, shard_rows, sharded_layout, wire_capacity, render_code_hash, wire_workspace_bytes)
from .poses import POSES, S0_POSE  # noqa: F401

# ray-step (sceneSDF) algorithmic FLOP per scene: SURVEY.md 8(d), DESIGN.md
FLOP_PER_EVAL = {"S0": 9, "T": 155, "O": 221, "OG": 221}
SCENES_DIR = __import__("os").path.join(__import__("os").path.dirname(__file__), "scenes")  # plugin examples
SCENE_FILES = {"S0": "sphere", "T": "template.frag", "O": "output_shader.frag", "OG": "output_shader_glass"}
