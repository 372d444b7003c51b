"""Numerics of the generic HIP kernels (csrc/kernels/gemm.hip, ops.hip) against
plain PyTorch fp32 references of the same op."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


def _act(z, act):
    return {"none": z, "relu": torch.relu(z), "sigmoid": torch.sigmoid(z), "tanh": torch.tanh(z),
            "gelu": torch.nn.functional.gelu(z)}[act]


@pytest.mark.parametrize("M,N,K", [(100, 100, 784), (100, 10, 100), (37, 129, 65), (256, 512, 1024),
                                   (1, 1, 1), (1000, 1, 1), (784, 100, 100)])
@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
def test_gemm_shapes_transposes(native, M, N, K, ta, tb):
    from distributed_tensorflow_example_amd import ops
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K)
    A = torch.randn((K, M) if ta else (M, K), generator=g)
    B = torch.randn((N, K) if tb else (K, N), generator=g)
    out = ops.matmul(A.cuda(), B.cuda(), ta, tb)
    ref = (A.t() if ta else A) @ (B.t() if tb else B)
    assert out.shape == ref.shape
    assert rel(out, ref) < 1e-2


@pytest.mark.parametrize("act", ["none", "relu", "sigmoid", "tanh", "gelu"])
@pytest.mark.parametrize("bf16_in", [False, True])
def test_gemm_bias_act_epilogue(native, act, bf16_in):
    from distributed_tensorflow_example_amd import ops
    g = torch.Generator().manual_seed(5)
    A, B, b = torch.randn(200, 300, generator=g), torch.randn(300, 130, generator=g), torch.randn(130, generator=g)
    dt = torch.bfloat16 if bf16_in else torch.float32
    out = ops.matmul(A.cuda().to(dt), B.cuda().to(dt), bias=b.cuda(), act=act)
    ref = _act(A.to(dt).float() @ B.to(dt).float() + b, act)
    assert rel(out, ref) < 1e-2


def test_gemm_alpha_beta_and_bf16_out(native):
    C = native
    A, B = torch.randn(64, 96).cuda(), torch.randn(96, 80).cuda()
    out = torch.randn(64, 80).cuda()
    o0 = out.clone()
    C.gemm(A, False, B, False, out, None, 0, 0.5, 2.0, None)
    assert rel(out, 0.5 * (A @ B) + 2.0 * o0) < 1e-2
    ob = torch.empty(64, 80, dtype=torch.bfloat16, device="cuda")
    C.gemm(A, False, B, False, ob, None, 0, 1.0, 0.0, None)
    assert rel(ob, A @ B) < 1e-2


@pytest.mark.parametrize("act", ["none", "relu", "sigmoid", "tanh", "gelu"])
def test_linear_act_autograd(native, act):
    from distributed_tensorflow_example_amd import ops
    torch.manual_seed(0)
    # operands pre-rounded to bf16 (what the MFMA GEMM consumes) so relu's
    # mask is the same on both sides; the fp32 reference then isolates the
    # kernel's own error
    x = torch.randn(100, 784).bfloat16().float().requires_grad_()
    w = torch.randn(784, 100).bfloat16().float().requires_grad_()
    b = torch.randn(100, requires_grad=True)
    y = _act(x @ w + b, act)
    gy = torch.randn_like(y)
    y.backward(gy)
    xg, wg, bg = [t.detach().cuda().requires_grad_() for t in (x, w, b)]
    yg = ops.linear_act(xg, wg, bg, act)
    yg.backward(gy.cuda())
    assert rel(yg, y) < 1e-2
    assert rel(xg.grad, x.grad) < 2e-2
    assert rel(wg.grad, w.grad) < 2e-2
    assert rel(bg.grad, b.grad) < 2e-2


@pytest.mark.parametrize("M,N", [(1000, 37), (4096, 512), (4096, 1), (4096, 256), (7, 12), (100000, 64), (33, 1028)])
def test_col_sum(native, M, N):
    X = torch.randn(M, N).cuda()
    out = torch.full((N,), float("nan"), device="cuda")
    native.col_sum(X, out)
    ref = X.cpu().double().sum(0).float()
    assert torch.allclose(out.cpu(), ref, atol=1e-4 * max(1.0, M ** 0.5), rtol=1e-4)


@pytest.mark.parametrize("dense", [False, True])
@pytest.mark.parametrize("naive", [False, True])
@pytest.mark.parametrize("B,Cn", [(100, 10), (7, 1000), (256, 3)])
def test_softmax_xent(native, dense, naive, B, Cn):
    from distributed_tensorflow_example_amd import ops
    torch.manual_seed(B + Cn)
    z = torch.randn(B, Cn) * 3
    lab = torch.randint(0, Cn, (B,))
    y = torch.nn.functional.one_hot(lab, Cn).float() if dense else lab
    zr = z.clone().requires_grad_()
    lr_ = torch.nn.functional.cross_entropy(zr, lab)
    lr_.backward()
    zg = z.cuda().requires_grad_()
    l = ops.softmax_xent(zg, y.cuda(), naive=naive)
    l.backward()
    assert abs(float(l) - float(lr_)) < 1e-4 * max(1.0, abs(float(lr_)))
    assert torch.allclose(zg.grad.cpu(), zr.grad, atol=1e-6)


def test_softmax_xent_correct_count(native):
    z = torch.randn(300, 10).cuda()
    lab = torch.randint(0, 10, (300,)).cuda()
    loss_rows = torch.empty(300, device="cuda")
    grad = torch.empty_like(z)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    native.softmax_xent(z, lab, None, loss_rows, grad, cnt, 1.0 / 300, False)
    assert int(cnt.item()) == int((z.argmax(1) == lab).sum())


@pytest.mark.parametrize("n", [1, 500, 4097])
def test_sigmoid_xent(native, n):
    from distributed_tensorflow_example_amd import ops
    torch.manual_seed(n)
    x = torch.randn(n, 1) * 4
    t = (torch.rand(n, 1) > 0.5).float()
    xr = x.clone().requires_grad_()
    ref = torch.nn.functional.binary_cross_entropy_with_logits(xr, t)
    ref.backward()
    xg = x.cuda().requires_grad_()
    l = ops.sigmoid_xent(xg, t.cuda())
    l.backward()
    assert abs(float(l) - float(ref)) < 1e-5 * max(1, abs(float(ref)))
    assert torch.allclose(xg.grad.cpu(), xr.grad, atol=1e-7)


def _bags(B, V, maxlen, seed):
    g = torch.Generator().manual_seed(seed)
    lens = torch.randint(0, maxlen + 1, (B,), generator=g)
    offsets = torch.zeros(B + 1, dtype=torch.int64)
    offsets[1:] = lens.cumsum(0)
    ids = torch.randint(0, V, (int(offsets[-1]),), generator=g)
    w = torch.rand(ids.numel(), generator=g)
    return ids, offsets, w


@pytest.mark.parametrize("D", [1, 16, 128, 33])
@pytest.mark.parametrize("mode", ["sum", "mean", "sqrtn"])
def test_embedding_bag_fwd_bwd(native, D, mode):
    from distributed_tensorflow_example_amd import ops
    V, B = 5000, 64
    ids, offsets, w = _bags(B, V, 40, D)
    W = torch.randn(V, D)
    Wr = W.clone().requires_grad_()
    ref = ops.embedding_bag(Wr, ids, offsets, w, mode)   # CPU path = torch oracle
    go = torch.randn_like(ref)
    ref.backward(go)
    Wg = W.cuda().requires_grad_()
    out = ops.embedding_bag(Wg, ids.cuda(), offsets.cuda(), w.cuda(), mode)
    out.backward(go.cuda())
    assert torch.allclose(out.cpu(), ref.detach(), atol=1e-4, rtol=1e-4)
    assert torch.allclose(Wg.grad.cpu(), Wr.grad, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("D", [1, 7, 64, 130])
def test_embedding_bag_bwd_sorted_hot_ids(native, D):
    """Zipf ids (one row hit thousands of times, runs crossing wave chunks) through
    the sorted-segment backward; a second table over the same ids reuses the plan."""
    from distributed_tensorflow_example_amd import ops
    import numpy as np
    rng = np.random.default_rng(D)
    B, nnz, V = 512, 24, 3000
    ids = torch.from_numpy((rng.zipf(1.1, B * nnz) - 1) % V).long()
    offsets = torch.arange(0, B * nnz + 1, nnz, dtype=torch.int64)
    w = torch.rand(ids.numel())
    W1, W2 = torch.randn(V, D), torch.randn(V, 3)
    go1, go2 = torch.randn(B, D), torch.randn(B, 3)
    refs = []
    for W, go in ((W1, go1), (W2, go2)):
        Wr = W.clone().requires_grad_()
        ops.embedding_bag(Wr, ids, offsets, w, "sum").backward(go)
        refs.append(Wr.grad)
    idc, offc, wc = ids.cuda(), offsets.cuda(), w.cuda()
    for (W, go), ref in zip(((W1, go1), (W2, go2)), refs):
        Wg = W.cuda().requires_grad_()
        ops.embedding_bag(Wg, idc, offc, wc, "sum").backward(go.cuda())
        assert rel(Wg.grad, ref) < 1e-5


@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_gemm_split_k_weight_grad(native, beta):
    """X^T dZ with K = batch 4096 and a 64 x 512 output: split over K, atomics into C."""
    C = native
    torch.manual_seed(3)
    X, dZ = torch.randn(4096, 64).cuda(), torch.randn(4096, 512).cuda()
    out = torch.randn(64, 512).cuda()
    o0 = out.clone()
    C.gemm(X, True, dZ, False, out, None, 0, 0.5, beta, None)
    # fp32 operands run on the exact-f32 MFMA path (no bf16 rounding)
    ref = (0.5 * (X.double().t() @ dZ.double()) + beta * o0.double()).float()
    assert rel(out, ref) < 1e-5


def test_embedding_bag_sgd_scatter(native):
    from distributed_tensorflow_example_amd import ops
    V, D, B = 1000, 1, 200
    ids, offsets, w = _bags(B, V, 30, 1)
    W = torch.randn(V)
    go = torch.randn(B, 1)
    ref = ops.embedding_bag_sgd_(W.clone(), ids, offsets, w, go, 0.5)
    got = ops.embedding_bag_sgd_(W.clone().cuda(), ids.cuda(), offsets.cuda(), w.cuda(), go.cuda(), 0.5)
    assert torch.allclose(got.cpu(), ref, atol=1e-5)


def test_bag_index_with_empty_bags(native):
    """bag_index (one binary search per CSR position) == repeat_interleave, empty bags included."""
    for seed, maxlen in ((1, 5), (2, 0), (3, 40)):
        ids, offsets, _ = _bags(300, 100, maxlen, seed)
        if ids.numel() == 0:
            offsets[-1] = 0
        ref = torch.repeat_interleave(torch.arange(300, dtype=torch.int32), offsets[1:] - offsets[:-1])
        out = torch.empty(ids.numel(), dtype=torch.int32, device="cuda")
        native.bag_index(offsets.cuda(), out)
        assert torch.equal(out.cpu(), ref)


def test_embedding_bag_sgd_identity_offsets(native):
    """offsets None: row i of the gradient goes to weight[ids[i]] (repeated ids accumulate)."""
    from distributed_tensorflow_example_amd import ops
    torch.manual_seed(4)
    V, D, n = 500, 24, 3000
    ids = torch.randint(0, V, (n,))
    g = torch.randn(n, D)
    W = torch.randn(V, D)
    ref = W.clone().index_add_(0, ids, g, alpha=-0.25)
    got = ops.embedding_bag_sgd_(W.clone().cuda(), ids.cuda(), None, None, g.cuda(), 0.25)
    assert torch.allclose(got.cpu(), ref, atol=1e-5)
    assert torch.allclose(ops.embedding_bag_sgd_(W.clone(), ids, None, None, g, 0.25), ref, atol=1e-5)


def test_argmax_correct(native):
    from distributed_tensorflow_example_amd import ops
    z = torch.randn(10000, 10)
    lab = torch.randint(0, 10, (10000,))
    assert int(ops.argmax_correct(z.cuda(), lab.cuda())) == int((z.argmax(1) == lab).sum())


def test_auc_histogram(native):
    from distributed_tensorflow_example_amd import ops
    n, nb = 20000, 200
    lab = (torch.rand(n) > 0.7).float()
    pred = torch.sigmoid(torch.randn(n) + 1.5 * lab)
    # predictions exactly on TF's fp32 thresholds and one ulp either side: the GPU
    # binary search must bin them like the CPU searchsorted (p > t is strict)
    t = ops.auc_thresholds(nb - 1)
    edge = torch.cat([t, torch.nextafter(t, torch.full_like(t, 2.0)), torch.nextafter(t, torch.full_like(t, -2.0))])
    pred[: edge.numel()] = edge
    pc, nc = torch.zeros(nb, dtype=torch.int64), torch.zeros(nb, dtype=torch.int64)
    ops.auc_histogram_(pred, lab, pc, nc)
    pg, ng = torch.zeros(nb, dtype=torch.int64, device="cuda"), torch.zeros(nb, dtype=torch.int64, device="cuda")
    ops.auc_histogram_(pred.cuda(), lab.cuda(), pg, ng)
    assert torch.equal(pg.cpu(), pc) and torch.equal(ng.cpu(), nc)
    # exact rank AUC
    order = pred.argsort()
    ranks = torch.empty(n)
    ranks[order] = torch.arange(1, n + 1).float()
    P = lab.sum()
    exact = float((ranks[lab > 0].sum() - P * (P + 1) / 2) / (P * (n - P)))
    assert abs(ops.auc_from_histograms(pg, ng) - exact) < 5e-3


@pytest.mark.parametrize("kind", ["sgd", "momentum", "nesterov", "adam", "adamw"])
@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
def test_fused_optimizers_match_cpu(native, kind, gdt):
    from distributed_tensorflow_example_amd import optim
    torch.manual_seed(1)
    shapes = [(784, 100), (100,), (100, 10), (10,), (5000,)]
    ps = [torch.randn(s) for s in shapes]

    def mk(params):
        if kind == "sgd":
            return optim.FusedSGD(params, 0.1)
        if kind in ("momentum", "nesterov"):
            return optim.FusedMomentum(params, 0.1, 0.9, nesterov=kind == "nesterov")
        if kind == "adam":
            return optim.FusedAdam(params, 0.01)
        return optim.FusedAdamW(params, 0.01, weight_decay=0.1)
    pc = [p.clone() for p in ps]
    pg = [p.clone().cuda() for p in ps]
    oc, og = mk(pc), mk(pg)
    for it in range(5):
        gs = [torch.randn(s).to(gdt) for s in shapes]
        oc.step(grads=[g.float() for g in gs], grad_scale=0.5)
        og.step(grads=[g.cuda() for g in gs], grad_scale=0.5)
    for a, b in zip(pg, pc):
        assert torch.allclose(a.cpu(), b, atol=2e-5, rtol=1e-5), (a.cpu() - b).abs().max()


def test_global_grad_norm(native):
    from distributed_tensorflow_example_amd import optim
    gs = [torch.randn(1000), torch.randn(77, 13), torch.randn(5)]
    n = optim.global_grad_norm([g.cuda() for g in gs])
    ref = math.sqrt(sum(float((g ** 2).sum()) for g in gs))
    assert abs(float(n) - ref) < 1e-4 * ref


def test_compat_mnist_graph_trains_on_gpu(native):
    """example.py-shaped graph through the compat layer on the GPU (MFMA linear)."""
    import numpy as np

    import distributed_tensorflow_example_amd.compat as tf
    from distributed_tensorflow_example_amd.data import mnist

    tf.reset_default_graph()
    ds = mnist.read_data_sets("/tmp/unused", one_hot=True, train_size=5000, test_size=1000)
    x = tf.placeholder(tf.float32, [None, 784])
    y_ = tf.placeholder(tf.float32, [None, 10])
    W1 = tf.Variable(tf.random_normal([784, 100], seed=1))
    W2 = tf.Variable(tf.random_normal([100, 10], seed=2))
    b1, b2 = tf.Variable(tf.zeros([100])), tf.Variable(tf.zeros([10]))
    a2 = tf.nn.sigmoid(tf.add(tf.matmul(x, W1), b1))
    y = tf.nn.softmax(tf.add(tf.matmul(a2, W2), b2))
    ce = tf.reduce_mean(-tf.reduce_sum(y_ * tf.log(y), reduction_indices=[1]))
    gs = tf.get_variable("global_step", [], initializer=tf.constant_initializer(0), trainable=False)
    train_op = tf.train.GradientDescentOptimizer(0.1).minimize(ce, global_step=gs)
    acc = tf.reduce_mean(tf.cast(tf.equal(tf.argmax(y, 1), tf.argmax(y_, 1)), tf.float32))
    with tf.Session() as sess:
        sess.run(tf.global_variables_initializer())
        first = None
        for _ in range(200):
            bx, by = ds.train.next_batch(100)
            _, c = sess.run([train_op, ce], {x: bx, y_: by})
            first = c if first is None else first
        a = sess.run(acc, {x: ds.test.images, y_: ds.test.labels})
        assert int(np.asarray(sess.run(gs))) == 200
    assert W1.value.is_cuda
    assert c < first and a > 0.4


@pytest.mark.parametrize("C,B", [(30522, 37), (10, 37), (1002, 37), (1001, 37), (30522, 300)])
def test_bf16_vocab_xent_with_bias(native, C, B):
    """bf16 vocab cross-entropy with the fused bias; its gradient from the in-tree
    column sums (16-byte / 4-byte row variants, several row slices) or torch's sum
    (odd vocab)."""
    from distributed_tensorflow_example_amd import ops
    torch.manual_seed(C)
    logits = (torch.randn(B, C) * 3).bfloat16()
    bias = torch.randn(C) * 0.5
    labels = torch.randint(0, C, (B,))
    lr_, br = logits.float().requires_grad_(), bias.clone().requires_grad_()
    ref = torch.nn.functional.cross_entropy(lr_ + br, labels)
    (ref * 3.0).backward()
    lg, bg = logits.cuda().requires_grad_(), bias.cuda().requires_grad_()
    out = ops.softmax_xent(lg, labels.cuda(), bias=bg)
    (out * 3.0).backward()                       # upstream scale is read on device
    assert abs(float(out) - float(ref)) < 1e-3 * max(1.0, abs(float(ref)))
    assert lg.grad.dtype == torch.bfloat16
    assert float((lg.grad.float().cpu() - lr_.grad).norm() / lr_.grad.norm()) < 1e-2
    assert float((bg.grad.cpu() - br.grad).norm() / br.grad.norm()) < 1e-2


@pytest.mark.gpu
def test_philox_normal_kernel_matches_cpu():
    """csrc/kernels/random.hip against the numpy Philox4x32-10 + Box-Muller of
    the same elements (fp32 transcendentals: a few ulp), incl. a strided shard."""
    from distributed_tensorflow_example_amd import ops

    for rows, dim, mul, add, seed in [(4097, 1, 1, 0, 123), (1000, 3, 4, 3, (1 << 40) + 5), (257, 64, 8, 1, 9)]:
        g = ops.philox_normal_(torch.empty(rows, dim, device="cuda"), mul, add, seed, 0.25, 1.5).cpu()
        c = ops.philox_normal_(torch.empty(rows, dim), mul, add, seed, 0.25, 1.5)
        assert torch.allclose(g, c, rtol=2e-6, atol=2e-6), (g - c).abs().max()


@pytest.mark.gpu
@pytest.mark.parametrize("W", [1, 3, 8])
def test_sparse_route_kernel_matches_torch(W):
    """csrc/kernels/sparse_route.hip (one-workgroup dedup + owner bucketing)
    against the torch emulation of the same outputs, Zipf ids incl. N < 1024
    and N spanning many per-thread chunks."""
    import numpy as np

    from distributed_tensorflow_example_amd import ops
    from distributed_tensorflow_example_amd.parallel.sharded_embedding import _route_static_torch

    rng = np.random.default_rng(W)
    for N in (1, 700, 20_000, 131_072):
        ids = torch.from_numpy(((rng.zipf(1.1, N) - 1) % 1_000_000).astype(np.int64)).cuda()
        sids, perm = torch.sort(ids.to(torch.int32))
        cap = N + 17
        got = ops._C().sparse_route(sids.contiguous(), perm, W, cap)
        want = _route_static_torch(sids.cpu(), perm.cpu(), W, cap)
        names = ["inv_sorted", "inverse", "uniq", "dest", "send"]
        for name, g, w_ in zip(names, got[:5], want):
            if W == 1 and name in ("dest", "send"):
                continue
            assert torch.equal(g.cpu(), w_.to(g.dtype)), (N, name)
        assert int(got[5].item()) == int(torch.unique(ids).numel())


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_bucket_pack_unpack_16bit(dt):
    """K16: DDP bucket -> bf16 / fp16 comm buffer with the 1/N scale folded in,
    and back, against torch's round-to-nearest-even cast (incl. a ragged tail)."""
    from distributed_tensorflow_example_amd import _native

    C = _native.load()
    for n in (8, 1000, (1 << 20) + 5):
        g = torch.randn(n, device="cuda") * 3
        c = torch.empty(n, dtype=dt, device="cuda")
        C.bucket_pack(g, c, 0.125)
        assert torch.equal(c, (g * 0.125).to(dt))
        out = torch.empty(n, device="cuda")
        C.bucket_unpack(c, out, 2.0)
        assert torch.equal(out, c.float() * 2.0)
    if dt == torch.bfloat16:        # the round-2 names stay bound
        C.bucket_pack_bf16(g, c, 1.0)
        assert torch.equal(c, g.to(dt))


@pytest.mark.gpu
@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
def test_gemm_fp32_operands_are_exact_f32(ta, tb):
    """fp32 x fp32 goes through the exact-f32 MFMA path (no bf16 rounding):
    relative error at fp32 summation level vs fp64, incl. ragged edges, bias +
    activation epilogue and the split-K (atomic) path."""
    from distributed_tensorflow_example_amd import ops

    g = torch.Generator(device="cpu").manual_seed(3)
    for M, N, K, act in [(37, 53, 29, "sigmoid"), (128, 64, 784, "none"), (100, 10, 100, "relu"), (64, 32, 4096, "none")]:
        a = torch.randn((K, M) if ta else (M, K), generator=g)
        b = torch.randn((N, K) if tb else (K, N), generator=g)
        bias = torch.randn(N, generator=g)
        got = ops.matmul(a.cuda(), b.cuda(), ta, tb, bias.cuda(), act).cpu().double()
        A = (a.t() if ta else a).double()
        Bm = (b.t() if tb else b).double()
        z = A @ Bm + bias.double()
        want = {"none": z, "relu": torch.relu(z), "sigmoid": torch.sigmoid(z)}[act]
        scale = (A.abs() @ Bm.abs()).max() + bias.abs().max()
        err = (got - want).abs().max() / scale
        assert err < 2e-6, (M, N, K, act, float(err))        # bf16 rounding would be ~4e-3


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["adagrad", "rmsprop"])
def test_fused_adagrad_rmsprop_match_cpu(kind):
    """multi_tensor_apply kinds 4/5 against the CPU math of the same optimizer."""
    from distributed_tensorflow_example_amd import optim

    torch.manual_seed(0)
    ps = [torch.randn(1000), torch.randn(37, 5)]
    gs = [[torch.randn_like(p) for p in ps] for _ in range(3)]
    mk = (lambda q: optim.FusedAdagrad(q, 0.05)) if kind == "adagrad" else \
        (lambda q: optim.FusedRMSProp(q, 0.01, 0.9, 0.5, 1e-10))
    pc = [p.clone() for p in ps]
    pg = [p.clone().cuda() for p in ps]
    oc, og = mk(pc), mk(pg)
    for step in gs:
        oc.step([g.clone() for g in step])
        og.step([g.clone().cuda() for g in step])
    for a, b in zip(pc, pg):
        assert torch.allclose(a, b.cpu(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("M,K", [(4096, 256), (256, 4096), (37, 5), (1000, 1)])
def test_gemm_fp32_matrix_vector(native, M, K, ta, tb):
    """N == 1 fp32 products (W&D head / its weight gradient) on the GEMV kernels."""
    torch.manual_seed(M + K)
    A = torch.randn(*((K, M) if ta else (M, K)), device="cuda")
    B = torch.randn(*((1, K) if tb else (K, 1)), device="cuda")
    a = (A.t() if ta else A).double()
    b = (B.t() if tb else B).double()
    for beta in (0.0, 1.0):
        C0 = torch.randn(M, 1, device="cuda")
        C = C0.clone()
        bias = torch.randn(1, device="cuda")
        native.gemm(A, ta, B, tb, C, bias=bias, act=0, alpha=0.5, beta=beta)
        ref = 0.5 * (a @ b) + bias.double() + beta * C0.double()
        assert torch.allclose(C.double(), ref, rtol=1e-5, atol=1e-4), (beta, float((C.double() - ref).abs().max()))
    if not ta:   # row form: any epilogue (activation + pre-activation output)
        C = torch.empty(M, 1, device="cuda")
        Z = torch.empty(M, 1, device="cuda")
        native.gemm(A, ta, B, tb, C, act=2, Z=Z)
        z = a @ b
        assert torch.allclose(Z.double(), z, rtol=1e-5, atol=1e-4)
        assert torch.allclose(C.double(), torch.sigmoid(z), rtol=1e-5, atol=1e-5)
