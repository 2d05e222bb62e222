"""librf.so loads without a GPU and exports every entry point declared in include/rf_api.h."""
import ctypes
import os
import re

from recommendflow_amd.runtime import lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols(header="rf_api.h"):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rf_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    assert "rf_fused_hash_embed_fwd" in syms and "rf_esim_soft_attention_fwd" in syms
    assert set(syms) == set(L.EXPORTED), set(syms) ^ set(L.EXPORTED)


def test_library_exports_every_declared_symbol():
    lib = L.load()
    for s in declared_symbols():
        assert hasattr(lib, s), s
    assert lib.rf_abi_version() == 1


def test_diag_header_exports():
    lib = L.load()
    syms = declared_symbols("rf_diag.h")
    assert set(syms) == set(L.DIAG_EXPORTED)
    for s in syms:
        assert hasattr(lib, s), s


def test_public_entry_rejects_ablation_bits():
    """Bits 12-14 change results: the production entry refuses them (validation precedes any HIP call)."""
    lib = L.load()
    for bit in (1 << 12, 1 << 13, 1 << 14, 1 << 10):
        rc = lib.rf_fused_hash_embed_fwd(None, 1, None, None, None, None, 4, None, 0, 10, 16, None, 0, 16, bit, None, None)
        assert rc == L.RF_EINVAL and b"flags" in lib.rf_last_error(), bit


def test_argument_errors_without_gpu():
    lib = L.load()
    # validation happens before any HIP call
    assert lib.rf_siphash_bucket(None, None, 4, 0, 0, 0, 1, None, None) == L.RF_EINVAL
    assert b"num_bins" in lib.rf_last_error()
    assert lib.rf_esim_soft_attention_fwd(None, None, 1, 1, 300, 128, 0, 128, None, 0, 0, None, None) == L.RF_EINVAL
    assert lib.rf_embedding_bag_fwd(None, 1, 1, 0, None, 0, 1, 4, 9, None, 0, 4, 0, None) == L.RF_EINVAL
    assert b"combiner" in lib.rf_last_error()
    assert lib.rf_bucketize_ws_bytes(1000, 8) >= 2 * 4 * 8 * 4


def test_product_path_has_no_oracle_import():
    pkg = os.path.join(ROOT, "recommendflow_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                text = open(os.path.join(dirpath, f)).read()
                assert "from oracle" not in text and "import oracle" not in text, f


def test_gemm_supported_applies_the_block_limit():
    """runtime.gemm.supported_gemm mirrors rf_gemm_f32's 2 GiB operand-block check per layout (meta tensors: no
    memory, no GPU): an m/n-contiguous operand's (K + 192) k-rows, a k-contiguous operand's 128 rows."""
    import torch

    from recommendflow_amd.runtime import gemm as G

    K = 4100
    a = torch.empty(K, 64, device="meta")
    wide = torch.empty(K, 131072, device="meta")      # (K + 192) * 131072 * 4 B >= 2 GiB
    narrow = torch.empty(K, 4096, device="meta")
    assert not G.supported_gemm(a, wide, trans_a=True, trans_b=False)
    assert not G.supported_gemm(a, wide[:, :4096], trans_a=True, trans_b=False)  # the view keeps the parent's ld
    assert G.supported_gemm(a, narrow, trans_a=True, trans_b=False)
    x = torch.empty(512, 1 << 22, device="meta")        # k-contiguous, 128 rows x 16 MiB = 2 GiB
    w = torch.empty(64, 1 << 22, device="meta")
    assert not G.supported_gemm(x, w, trans_b=True)
    assert G.supported_gemm(x[:, : 1 << 20].contiguous(), w[:, : 1 << 20].contiguous(), trans_b=True)
    assert not G.supported_gemm(torch.empty(64, 30, device="meta"), torch.empty(16, 30, device="meta"), trans_b=True)
