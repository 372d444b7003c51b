"""The BERT-base GEMM engine table (ops/big_gemm.py): under 'auto' the listed
products take the table's engine without timing, other shapes are timed, and
DTF_BIG_GEMM_TABLE=0 / another policy bypass it."""


def test_fixed_table_lookup(monkeypatch):
    from distributed_tensorflow_example_amd.ops import big_gemm

    monkeypatch.setattr(big_gemm, "_POLICY", "auto")
    monkeypatch.setattr(big_gemm, "_TABLE_ON", True)
    assert big_gemm._fixed(("dw", 3072, 768, 16384)) is False      # FFN1 weight gradient: hipBLASLt
    assert big_gemm._fixed(("gelu_aux", 16384, 3072, 768)) is True  # fused GELU forward epilogue
    assert big_gemm._fixed(("fwd", 1024, 768, 768)) is None         # not listed: timed
    monkeypatch.setattr(big_gemm, "_TABLE_ON", False)
    assert big_gemm._fixed(("dw", 3072, 768, 16384)) is None
    monkeypatch.setattr(big_gemm, "_TABLE_ON", True)
    monkeypatch.setattr(big_gemm, "_POLICY", "always")
    assert big_gemm._fixed(("dw", 3072, 768, 16384)) is None


def test_table_covers_every_bert_base_linear_product():
    from distributed_tensorflow_example_amd.ops import big_gemm

    T, H, F = 16384, 768, 3072
    prods = []
    for n_in, n_out in ((H, 3 * H), (H, H), (H, F), (F, H)):     # qkv, attention out, FFN1, FFN2
        prods += [("fwd", T, n_out, n_in), ("dx", T, n_in, n_out), ("dw", n_out, n_in, T)]
    missing = [p for p in prods if p not in big_gemm._TABLE]
    assert missing == [], missing
