"""K27 fused LSTM: fragment packing (CPU), nn.LSTM parity of the module (CPU), HIP kernels vs the
fp32 oracle (GPU)."""
import pytest
import torch

from avenir_amd.ops import rnn
from avenir_amd import _native


@pytest.mark.parametrize("H,I", [(20, 5), (64, 64), (100, 100), (37, 128)])
def test_pack_weights_fragment_maps(H, I):
    torch.manual_seed(0)
    Whh, Wih = torch.randn(4 * H, H), torch.randn(4 * H, I)
    fwd, bwd = rnn.pack_weights(Wih, Whh, H)
    HP, IP = rnn.padded_hidden(H), rnn.padded_hidden(I)
    KS, NW, KT = HP // 32, HP // 16, (HP + IP) // 32
    assert fwd.shape == (NW, 4, KT, 4, 16, 8) and bwd.shape == (NW, 4 * KS, 4, 16, 8)
    fwd = fwd.float().reshape(NW, 4, KT, 64, 8)
    bwd = bwd.float().reshape(NW, 4 * KS, 64, 8)
    Hb, Ib = Whh.to(torch.bfloat16).float(), Wih.to(torch.bfloat16).float()

    def wcat(r, c):  # padded [W_hh | W_ih] element, rows gate-major
        g, u = divmod(r, HP)
        if u >= H:
            return 0.0
        if c < HP:
            return Hb[g * H + u, c].item() if c < H else 0.0
        return Ib[g * H + u, c - HP].item() if c - HP < I else 0.0

    g_ = torch.Generator().manual_seed(1)
    for _ in range(300):
        w, g, ks, lane, j = (int(torch.randint(0, n, (1,), generator=g_)) for n in (NW, 4, KT, 64, 8))
        col, q = lane & 15, lane >> 4
        assert fwd[w, g, ks, lane, j].item() == wcat(g * HP + 16 * w + col, 32 * ks + 8 * q + j)
        s = int(torch.randint(0, 4 * KS, (1,), generator=g_))
        gg, kk = divmod(s, KS)
        assert bwd[w, s, lane, j].item() == wcat(gg * HP + 32 * kk + 8 * q + j, 16 * w + col)


@pytest.mark.parametrize("H", [20, 64, 100, 128])
def test_pack_weights_f32_fragment_maps(H):
    torch.manual_seed(1)
    Whh = torch.randn(4 * H, H)
    fwd, bwd = rnn.pack_weights_f32(Whh, H)
    HP = rnn.padded_hidden(H)
    NW, KS4 = HP // 16, HP // 4
    assert fwd.shape == (NW, 4, KS4, 64) and bwd.shape == (NW, HP, 64)

    def w(r, c):  # padded W_hh, rows gate-major g*HP + u
        g, u = divmod(r, HP)
        return Whh[g * H + u, c].item() if u < H and c < H else 0.0

    g_ = torch.Generator().manual_seed(2)
    for _ in range(400):
        wv, g, s, lane = (int(torch.randint(0, n, (1,), generator=g_)) for n in (NW, 4, KS4, 64))
        col, q = lane & 15, lane >> 4
        assert fwd[wv, g, s, lane].item() == w(g * HP + 16 * wv + col, 4 * s + q)
        k = int(torch.randint(0, HP, (1,), generator=g_))
        assert bwd[wv, k, lane].item() == w(4 * k + q, 16 * wv + col)


@pytest.mark.gpu
@pytest.mark.parametrize("H,I", [(20, 3), (100, 1), (100, 100), (128, 7)])
def test_lstm_pack_f32_kernel_matches_python_packers(cuda, H, I):
    """rnn_f32.hip lstm_pack_f32_kernel (one launch) == the documented fragment maps + kernel gate
    order + the summed biases."""
    torch.manual_seed(H + I)
    w_ih, w_hh = torch.randn(4 * H, I, device=cuda), torch.randn(4 * H, H, device=cuda)
    b_ih, b_hh = torch.randn(4 * H, device=cuda), torch.randn(4 * H, device=cuda)
    frag, frag_t, wihk, biask, wx = _native.C().lstm_pack_f32(w_ih, w_hh, b_ih, b_hh)
    f_ref, ft_ref = rnn.pack_weights_f32(w_hh, H)
    assert torch.equal(frag, f_ref) and torch.equal(frag_t, ft_ref)
    assert torch.equal(wihk, rnn.to_kernel_order(w_ih, H))
    assert torch.equal(biask, rnn.to_kernel_order(b_ih + b_hh, H))
    _, _, _, b1, _ = _native.C().lstm_pack_f32(w_ih, w_hh, None, b_hh)
    assert torch.equal(b1, rnn.to_kernel_order(b_hh, H))
    if I <= 8:   # W_ih fragments of the in-kernel projection: lane q*16 + col of k-step s holds W_ih[g*H + 16w + col, 4s + q]
        HP = rnn.padded_hidden(H)
        wp = torch.zeros((4, HP, 8), device=cuda)
        wp[:, :H, :I] = w_ih.view(4, H, I)
        ref = wp.view(4, HP // 16, 16, 2, 4).permute(1, 0, 3, 4, 2).reshape(HP // 16, 4, 2, 64)
        assert torch.equal(wx, ref)
    else:
        assert wx.numel() == 0


@pytest.mark.gpu
def test_fused_lstm_module_matches_torch_lstm_gpu(cuda):
    """The fp32 module (split biases, torch-order dz, forward-written h_{t-1} rows) against
    torch.nn.LSTM on the GPU: outputs and every parameter's gradient."""
    torch.manual_seed(0)
    ref = torch.nn.LSTM(5, 100, 2, batch_first=True).to(cuda)
    mine = rnn.FusedLSTM(5, 100, 2).to(cuda)
    mine.load_state_dict(ref.state_dict())
    x = torch.randn(300, 5, 5, device=cuda)
    h0, c0 = torch.randn(2, 300, 100, device=cuda), torch.randn(2, 300, 100, device=cuda)
    o1, (h1, c1) = ref(x, (h0, c0))
    o2, (h2, c2) = mine(x, (h0, c0))
    torch.testing.assert_close(o2, o1, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(c2, c1, atol=1e-4, rtol=1e-4)
    (o1.square().sum() + c1.sum()).backward()
    (o2.square().sum() + c2.sum()).backward()
    for (n, p1), p2 in zip(ref.named_parameters(), mine.parameters()):
        rel = (p2.grad - p1.grad).norm() / p1.grad.norm()
        assert rel.item() < 1e-4, (n, rel.item())


def test_fused_lstm_module_matches_torch_lstm_cpu():
    torch.manual_seed(0)
    ref = torch.nn.LSTM(6, 10, 2, batch_first=True)
    mine = rnn.FusedLSTM(6, 10, 2)
    mine.load_state_dict(ref.state_dict())
    x = torch.randn(5, 7, 6)
    h0, c0 = torch.randn(2, 5, 10), torch.randn(2, 5, 10)
    o1, (h1, c1) = ref(x, (h0, c0))
    o2, (h2, c2) = mine(x, (h0, c0))
    torch.testing.assert_close(o2, o1, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(h2, h1, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(c2, c1, atol=1e-5, rtol=1e-5)
    (o1.square().sum() + c1.sum()).backward()
    (o2.square().sum() + c2.sum()).backward()
    for (n, p1), p2 in zip(ref.named_parameters(), mine.parameters()):
        torch.testing.assert_close(p2.grad, p1.grad, atol=1e-4, rtol=1e-4, msg=n)


def _oracle(x, w_ih, w_hh, b, h0, c0):
    x, w_ih, w_hh, b = (t.detach().double().requires_grad_() for t in (x, w_ih, w_hh, b))
    h0 = h0.detach().double().requires_grad_()
    c0 = c0.detach().double().requires_grad_()
    hs, (h, c) = rnn.lstm_reference(x, w_ih, w_hh, b, h0, c0)
    return (x, w_ih, w_hh, b, h0, c0), hs, h, c


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["bf16", "fp32"])
@pytest.mark.parametrize("B,T,I,H", [(37, 5, 3, 20), (50, 4, 3, 37), (1000, 5, 8, 100), (9000, 6, 16, 64), (20000, 3, 4, 128),
                                     (3000, 4, 64, 48), (700, 3, 128, 128), (500, 2, 100, 64)])
def test_fused_lstm_kernels_vs_fp32_oracle(cuda, B, T, I, H, prec):
    torch.manual_seed(B)
    k = 1.0 / H ** 0.5
    x = torch.randn(B, T, I, device=cuda)
    w_ih = (torch.rand(4 * H, I, device=cuda) * 2 - 1) * k
    w_hh = (torch.rand(4 * H, H, device=cuda) * 2 - 1) * k
    b = (torch.rand(4 * H, device=cuda) * 2 - 1) * k
    h0 = torch.randn(B, H, device=cuda) * 0.5
    c0 = torch.randn(B, H, device=cuda) * 0.5
    leaves = [t.clone().requires_grad_() for t in (x, w_ih, w_hh, b, h0, c0)]
    hs, h, c = rnn.lstm_layer(*leaves, precision=prec)
    assert hs.shape == (B, T, H)
    ins, hs_r, h_r, c_r = _oracle(x, w_ih, w_hh, b, h0, c0)
    # bf16: bf16 recurrent operands, fp32 accumulation / gate math; fp32: f32 MFMA chains throughout
    tol_h, tol_c, tol_g = (2e-2, 3e-2, 3e-2) if prec == "bf16" else (2e-5, 3e-5, 2e-5)
    assert (hs.double() - hs_r).abs().max().item() < tol_h
    assert (c.double() - c_r).abs().max().item() < tol_c
    gy = torch.randn_like(hs)
    gc = torch.randn_like(c)
    (hs * gy).sum().backward(retain_graph=True)
    (c * gc).sum().backward()
    ((hs_r * gy.double()).sum() + (c_r * gc.double()).sum()).backward()
    for name, mine, ref in zip(["x", "w_ih", "w_hh", "b", "h0", "c0"], leaves, ins):
        g1, g2 = mine.grad.double(), ref.grad
        rel = (g1 - g2).norm() / g2.norm().clamp_min(1e-12)
        assert rel.item() < tol_g, (name, rel.item())


@pytest.mark.gpu
def test_fused_lstm_network_trains(cuda):
    from avenir_amd.nn.sequence import LstmNetwork
    torch.manual_seed(0)
    n, T = 4096, 5
    x = torch.rand(n, T, 1, device=cuda)
    y = (x.sum(dim=(1, 2)) > T / 2).float()
    net = LstmNetwork(1, 100, 1, num_layers=2, seq_len=T, batch_size=256, lr=0.01, num_iter=60, device=cuda)
    assert isinstance(net.lstm, rnn.FusedLSTM)
    net.fit(x, y)
    assert net.losses[-1] < 0.6 * net.losses[0]


@pytest.mark.parametrize("H", [20, 64, 100, 128])
def test_kernel_gate_order_roundtrip(H):
    HP = rnn.padded_hidden(H)
    w = torch.randn(4 * H, 3)
    k = rnn.to_kernel_order(w, H)
    assert k.shape == (4 * HP, 3)
    for kc in range(4 * HP):
        wv, g, i = kc // 64, (kc % 64) // 16, kc % 16
        u = 16 * wv + i
        expect = w[g * H + u] if u < H else torch.zeros(3)
        assert torch.equal(k[kc], expect)
    _, _, inv = rnn.kernel_gate_order(H, w.device)
    assert torch.equal(k.index_select(0, inv), w)


@pytest.mark.gpu
def test_lstm_network_graph_matches_eager(cuda):
    """The captured HIP-graph train step (warm-up state restored) trains exactly like eager."""
    from avenir_amd.nn.sequence import LstmNetwork
    torch.manual_seed(0)
    x = torch.rand(512, 5, 3, device=cuda)
    y = (x.sum(dim=(1, 2)) > 7.5).float()
    nets = []
    for graph in (False, True):
        torch.manual_seed(1)
        net = LstmNetwork(3, 40, 1, num_layers=2, seq_len=5, batch_size=128, lr=0.01, num_iter=4, device=cuda,
                          graph=graph)
        # same optimiser arithmetic on both sides (capturable Adam keeps its step count on device)
        net.optimizer = torch.optim.Adam(net.parameters(), lr=0.01, capturable=True)
        net.fit(x, y)
        nets.append(net)
    torch.testing.assert_close(torch.tensor(nets[1].losses), torch.tensor(nets[0].losses), rtol=1e-4, atol=1e-5)
    for p0, p1 in zip(nets[0].parameters(), nets[1].parameters()):
        torch.testing.assert_close(p1, p0, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
def test_fused_fp32_lstm_loss_curve_equals_nn_lstm(cuda):
    """The default fp32 fused kernels against an fp32 torch.nn.LSTM (MIOpen) from the same weights
    and batches: the training loss curves agree at fp32 tolerance over all steps.  Plain SGD: Adam
    divides by the running gradient RMS, which turns last-bit differences between two correct fp32
    implementations into visibly different trajectories once the gradients become small."""
    from avenir_amd.nn.sequence import LstmNetwork
    torch.manual_seed(0)
    n, T = 2048, 5
    x = torch.rand(n, T, 2, device=cuda)
    y = ((x[..., 0] - x[..., 1]).sum(1) > 0).float()
    curves = {}
    for kind in ("fused", "nn"):
        torch.manual_seed(3)
        net = LstmNetwork(2, 100, 1, num_layers=2, seq_len=T, batch_size=256, lr=0.005, num_iter=40, device=cuda,
                          graph=False)
        assert net.lstm.precision == "fp32"
        if kind == "nn":
            ref = torch.nn.LSTM(2, 100, 2, batch_first=True).to(cuda)
            ref.load_state_dict(net.lstm.state_dict())
            net.lstm = ref
        net.optimizer = torch.optim.SGD(net.parameters(), lr=2.0)
        torch.manual_seed(11)
        net.fit(x, y)
        curves[kind] = torch.tensor(net.losses)
    a, b = curves["fused"], curves["nn"]
    assert a.shape == b.shape and b[-10:].mean() < 0.6 * b[0]
    assert float(((a - b).abs() / b.abs()).max()) < 1e-3, (a, b)
    assert float(((a[:6] - b[:6]).abs() / b[:6].abs()).max()) < 1e-4, (a, b)


@pytest.mark.gpu
def test_fused_lstm_loss_curve_matches_fp32_nn_lstm(cuda):
    """Mixed-precision fused kernels vs an fp32 torch.nn.LSTM from the same initialisation and the
    same batches: the training loss curves agree within bf16 tolerance (the reference trains fp32)."""
    from avenir_amd.nn.sequence import LstmNetwork
    torch.manual_seed(0)
    n, T = 2048, 5
    x = torch.rand(n, T, 2, device=cuda)
    y = ((x[..., 0] - x[..., 1]).sum(1) > 0).float()
    curves = {}
    for prec in ("bf16", "fp32"):
        torch.manual_seed(3)
        net = LstmNetwork(2, 100, 1, num_layers=2, seq_len=T, batch_size=256, lr=0.005, num_iter=40, device=cuda,
                          graph=False, precision="bf16" if prec == "bf16" else "fp32")
        if prec == "fp32":      # a plain fp32 nn.LSTM with the same weights (state dicts are compatible)
            ref = torch.nn.LSTM(2, 100, 2, batch_first=True).to(cuda)
            ref.load_state_dict(net.lstm.state_dict())
            net.lstm = ref
            net.optimizer = torch.optim.Adam(net.parameters(), lr=0.005)
        else:
            net.optimizer = torch.optim.Adam(net.parameters(), lr=0.005)
        torch.manual_seed(11)                  # same batch order
        net.fit(x, y)
        curves[prec] = torch.tensor(net.losses)
    a, b = curves["bf16"], curves["fp32"]
    assert a.shape == b.shape and b[-10:].mean() < 0.3 * b[0]
    # step by step while the loss is large (measured: <= 0.3 % rel over the first 6 steps); once
    # the loss is small, SGD noise dominates and only the level of the curve is compared
    assert float(((a[:6] - b[:6]).abs() / b[:6].abs()).max()) < 0.01, (a, b)
    for w in range(0, a.numel(), 10):
        r = float(a[w:w + 10].mean() / b[w:w + 10].mean())
        assert 0.5 < r < 2.0, (w, r, a, b)


def test_fp32_precision_option_cpu():
    m = rnn.FusedLSTM(3, 8, 2, precision="fp32")
    x = torch.randn(4, 5, 3)
    ref = torch.nn.LSTM(3, 8, 2, batch_first=True)
    ref.load_state_dict(m.state_dict())
    torch.testing.assert_close(m(x)[0], ref(x)[0], rtol=1e-5, atol=1e-6)
    with pytest.raises(ValueError):
        rnn.FusedLSTM(3, 8, precision="fp16")
    assert rnn.FusedLSTM(3, 8).precision == "fp32"          # the reference's numerics by default
