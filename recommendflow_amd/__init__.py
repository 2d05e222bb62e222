"""recommendflow_amd — MI355X-native (gfx950) sparse-feature embedding + attention-ranking hot path of
mechsihao/RecommendFlow, behind the reference's own operator API (backend.layers / backend.encoder /
backend.blocks / config_parser). Kernels live in csrc/ (librf.so, C ABI: include/rf_api.h)."""
__version__ = "0.1.0"
