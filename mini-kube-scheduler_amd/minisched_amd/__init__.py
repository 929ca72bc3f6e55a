"""minisched_amd — MI355X scheduling-cycle engine (Python side of the C ABI).

The product is libminisched_gpu.so (HIP, gfx950). This package only binds it
(`_lib`), encodes v1 objects into flat records (`encode`), generates the
BASELINE.json synthetic clusters (`synth`) and runs the node-sharded
multi-GPU combine over torch.distributed (`sharded`).
"""
from ._lib import (  # noqa: F401
    CODE_ERROR,
    CODE_SUCCESS,
    CODE_UNSCHEDULABLE,
    MASK_NODE_RESOURCES_FIT,
    MASK_NODE_UNSCHEDULABLE,
    MODE_BATCHED,
    MODE_SEQUENTIAL,
    NODE_REC,
    PLUGINS_NU_NN,
    PLUGINS_NU_NRF_NN_LA,
    POD_REC,
    RESULT,
    Engine,
    MSError,
    device_count,
    load,
)
