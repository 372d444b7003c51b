"""HIP row-sparse optimizer kernel (csrc/kernels/sparse_optim.hip) and the
shard-wide fused Adam of a sharded table, on the GPU, against the dense
NumPy model of TensorFlow's sparse-apply semantics."""
import numpy as np
import pytest
import torch

from test_sparse_optim_cpu import HP, make_steps, reference, run_table

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", ["momentum", "adagrad", "rmsprop", "adam"])
@pytest.mark.parametrize("D", [1, 6, 16])
def test_sparse_rule_gpu_matches_tf_model(native, kind, D):
    rows, lr = 5000, 0.05
    steps = make_steps(rows, D, 2048, 4, seed=D)
    t, t0 = run_table(kind, rows, D, steps, lr, device="cuda")
    var, a, b = reference(kind, t0, steps, lr, HP[kind])
    np.testing.assert_allclose(t.local.cpu().numpy(), var, rtol=1e-4, atol=1e-5)
    first = {"momentum": "Momentum", "adagrad": "Adagrad", "rmsprop": "RMSProp", "adam": "Adam"}[kind]
    np.testing.assert_allclose(t.slots[first].cpu().numpy(), a, rtol=1e-4, atol=1e-6)
    assert float(t._gacc.abs().max()) == 0.0


@pytest.mark.parametrize("kind", ["adagrad", "adam"])
def test_voided_step_gpu(native, kind):
    rows, D, lr = 3000, 4, 0.05
    steps = make_steps(rows, D, 512, 3, seed=5)
    t, t0 = run_table(kind, rows, D, steps, lr, device="cuda", void_step=1)
    var, _, _ = reference(kind, t0, [steps[0], steps[2]], lr, HP[kind])
    np.testing.assert_allclose(t.local.cpu().numpy(), var, rtol=1e-4, atol=1e-5)


def test_kernel_rejects_bad_shapes(native):
    table = torch.zeros(10, 4, device="cuda")
    with pytest.raises(RuntimeError):
        native.sparse_rows_apply(table, None, None, torch.zeros(3, dtype=torch.int64, device="cuda"),
                                 torch.zeros(3, 5, device="cuda"), 0, 0.1)
    with pytest.raises(RuntimeError):     # adagrad needs its accumulator
        native.sparse_rows_apply(table, None, None, torch.zeros(3, dtype=torch.int64, device="cuda"),
                                 torch.zeros(3, 4, device="cuda"), 4, 0.1)
