"""Neural models: MLP (layer spec, graphs), LSTM, autoencoder, RBM imputation, DQN pricing."""
import pytest
import torch

from avenir_amd.nn import (AutoEncoder, DQNAgent, FeedForwardNetwork, LstmNetwork, PolicyServer, PricingEnv,
                           RestrictedBoltzmannMachine, parse_layer_spec)
from avenir_amd.utils.config import Configuration


def _xor_data(n=2000, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand((n, 2), generator=g) * 2 - 1
    y = ((x[:, 0] * x[:, 1]) > 0).long()
    return x, y


def test_layer_spec():
    s = parse_layer_spec("8:relu:true:false:0.1,4:tanh:true:true:0,1:none:false:false:0", 5)
    kinds = [type(m).__name__ for m in s]
    assert kinds == ["Linear", "BatchNorm1d", "ReLU", "Dropout", "Linear", "Tanh", "BatchNorm1d", "Linear"]
    with pytest.raises(ValueError):
        parse_layer_spec("8:relu", 3)


def test_mlp_classifier_and_checkpoint(tmp_path):
    x, y = _xor_data()
    m = FeedForwardNetwork("16:relu:false:false:0,16:relu:false:false:0,2:none:false:false:0", 2, loss="ce",
                           optimizer="adam", lr=0.01, batch_size=64, num_iter=60, device="cpu")
    m.fit(x, y, track_interval=10)
    acc = m.evaluate_model(x, y, "accuracy")
    assert acc > 0.95
    assert m.errors[-1] < m.errors[0]
    p = tmp_path / "mlp.pt"
    m.save(p)
    m2 = FeedForwardNetwork("16:relu:false:false:0,16:relu:false:false:0,2:none:false:false:0", 2, loss="ce",
                            device="cpu")
    m2.restore(p)
    assert torch.equal(m2.predict(x, "binary"), m.predict(x, "binary"))


def test_mlp_from_config(tmp_path):
    rows = []
    g = torch.Generator().manual_seed(1)
    X = torch.rand((500, 3), generator=g)
    t = X @ torch.tensor([1.0, -2.0, 0.5]) + 0.3
    for i in range(500):
        rows.append(f"id{i},{X[i, 0]:.5f},{X[i, 1]:.5f},{X[i, 2]:.5f},{t[i]:.5f}")
    f = tmp_path / "train.csv"
    f.write_text("\n".join(rows))
    conf = Configuration({"train.data.fields": "1,2,3,4", "train.data.feature.fields": "0,1,2",
                          "train.data.out.fields": "3", "train.layer.data": "8:relu:false:false:0,1:none:false:false:0",
                          "train.optimizer": "adam", "train.opt.learning.rate": "0.01", "train.batch.size": "32",
                          "train.num.iterations": "80", "train.lossFn": "mse", "common.device": "cpu"}, {})
    m = FeedForwardNetwork.from_config(conf)
    x, y = m.prep_data(f)
    assert x.shape == (500, 3) and y.shape == (500, 1)
    m.fit(x, y)
    assert m.evaluate_model(x, y, "rmse") < 0.15


def test_lstm_seq_to_one_and_seq():
    g = torch.Generator().manual_seed(0)
    n, S = 600, 5
    seq = torch.rand((n, S * 1), generator=g)
    y = (seq.sum(1) > S / 2).float()
    m = LstmNetwork(1, 16, 1, seq_len=S, batch_size=32, out_activation="sigmoid", loss="bce", lr=0.01, num_iter=40,
                    device="cpu")
    x = m.to_sequences(seq)
    m.fit(x, y)
    acc = float((m.predict(x, "binary") == y.long()).float().mean())
    assert acc > 0.9
    ms = LstmNetwork(1, 8, 1, seq_len=S, out_sequence=True, out_activation=None, lr=0.01, num_iter=5, device="cpu")
    out = ms.predict(ms.to_sequences(seq))
    assert out.shape == (n, S, 1)


def test_autoencoder_anomaly():
    g = torch.Generator().manual_seed(0)
    z = torch.randn((2000, 2), generator=g)
    A = torch.randn((2, 8), generator=g)
    x = z @ A + 0.01 * torch.randn((2000, 8), generator=g)
    ae = AutoEncoder(8, [4, 2], ["tanh", None], ["tanh", None], lr=0.01, batch_size=128, num_iter=60, device="cpu")
    ae.fit(x)
    assert ae.losses[-1] < ae.losses[0] * 0.2
    assert ae.encode(x).shape == (2000, 2)
    out = torch.randn((20, 8), generator=g) * 3
    assert float(ae.reconstruction_error(out).mean()) > 3 * float(ae.reconstruction_error(x).mean())


def test_rbm_imputation():
    g = torch.Generator().manual_seed(0)
    # two binary prototypes with noise
    proto = torch.tensor([[1, 1, 1, 1, 0, 0, 0, 0], [0, 0, 0, 0, 1, 1, 1, 1]], dtype=torch.float32)
    lab = torch.randint(0, 2, (1000,), generator=g)
    x = proto[lab]
    flip = torch.rand(x.shape, generator=g) < 0.03
    x = torch.where(flip, 1 - x, x)
    rbm = RestrictedBoltzmannMachine(8, 6, lr=0.05, batch_size=10, num_iter=20, device="cpu").fit(x)
    miss = torch.zeros_like(x, dtype=torch.bool)
    miss[:, 0] = True
    miss[:, 5] = True
    imp = rbm.impute(x, miss, n_iter=60)
    truth = proto[lab]
    acc = float((imp[:, [0, 5]] == truth[:, [0, 5]]).float().mean())
    assert acc > 0.9


def test_dqn_pricing_learns():
    torch.manual_seed(0)          # the agent's exploration / init draw from the global generator
    env = PricingEnv(64, device="cpu", seed=0)
    s = env.reset()
    assert s.shape == (64, 41)
    agent = DQNAgent(env, lr=0.002, gamma=0.8, batch=256, hiddens=(64, 64), eps_decay_steps=300, target_sync=50)
    base = agent.evaluate()
    agent.train(iterations=25)
    after = agent.evaluate()
    assert after > base * 0.98     # learned policy is at least as good as the initial greedy policy
    srv = PolicyServer(agent)
    prices = srv.get_price(env.reset()[:3])
    assert len(prices) == 3 and all(400 <= p < 500 for p in prices)


@pytest.mark.gpu
def test_mlp_graph_capture_on_gpu(cuda):
    x, y = _xor_data(4096)
    m = FeedForwardNetwork("32:relu:false:false:0,32:relu:false:false:0,2:none:false:false:0", 2, loss="ce",
                           optimizer="adam", lr=0.01, batch_size=256, num_iter=40, device="cuda", graph=True)
    m.fit(x, y)
    assert m.evaluate_model(x, y, "accuracy") > 0.95
    lstm = LstmNetwork(1, 16, 1, seq_len=5, batch_size=64, loss="bce", lr=0.01, num_iter=5, device="cuda")
    seq = torch.rand((256, 5))
    lstm.fit(lstm.to_sequences(seq), (seq.sum(1) > 2.5).float())
    assert lstm.predict(lstm.to_sequences(seq)).device.type == "cuda"


def test_fused_layer_spec_keeps_indices():
    s = parse_layer_spec("8:relu:false:false:0,4:sigmoid:false:false:0.2,1:none:false:false:0", 5)
    kinds = [type(m).__name__ for m in s]
    assert kinds == ["FusedLinear", "Identity", "FusedLinear", "Identity", "Dropout", "Linear"]
    ref = parse_layer_spec("8:relu:false:false:0,4:sigmoid:false:false:0.2,1:none:false:false:0", 5, fuse=False)
    assert list(s.state_dict().keys()) == list(ref.state_dict().keys())
    ref.load_state_dict(s.state_dict())
    s.eval(), ref.eval()
    x = torch.randn(7, 5)
    assert torch.allclose(s(x), ref(x), atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("act", ["none", "relu", "sigmoid", "tanh", "leakyRelu", "elu"])
@pytest.mark.parametrize("M,K,N", [(37, 5, 3), (300, 64, 130), (1025, 33, 64), (20000, 48, 64), (20000, 200, 96)])
def test_linear_act_kernel_matches_torch(cuda, act, M, K, N):
    from avenir_amd.ops.mlp_ops import _act_torch, ACT_CODES, linear_act
    g = torch.Generator().manual_seed(M + N)
    x = torch.randn(M, K, generator=g, dtype=torch.float64)
    W = torch.randn(N, K, generator=g, dtype=torch.float64) / K ** 0.5
    b = torch.randn(N, generator=g, dtype=torch.float64)
    gy = torch.randn(M, N, generator=g, dtype=torch.float64)
    xr, Wr, br = (t.clone().requires_grad_() for t in (x, W, b))
    yr = _act_torch(torch.nn.functional.linear(xr, Wr, br), ACT_CODES[act])
    yr.backward(gy)
    xg, Wg, bg = (t.float().to(cuda).requires_grad_() for t in (x, W, b))
    yg = linear_act(xg, Wg, bg, act)
    yg.backward(gy.float().to(cuda))
    assert torch.allclose(yg.detach().cpu().double(), yr.detach(), atol=1e-4, rtol=1e-4)
    # the kernel's derivative is taken from its own stored output, so at a kink (relu / leaky relu
    # / elu at z ~ 0) the fp64 forward's decision is not the reference: in any split-bf16 mode a
    # few of 1.3 M pre-activations within the GEMM's error of 0 land on the other side.  The
    # gradient oracle is the fp64 backward of that same decision (dZ from the GPU's y).
    y = yg.detach().cpu().double()
    code = ACT_CODES[act]
    dact = {0: torch.ones_like(y), 1: (y > 0).double(), 2: y * (1 - y), 3: 1 - y * y,
            4: torch.where(y > 0, 1.0, 0.01).double(), 5: torch.where(y > 0, 1.0, y + 1)}[code]
    dz = gy * dact
    for a, r in ((xg.grad, dz @ W), (Wg.grad, dz.t() @ x), (bg.grad, dz.sum(0))):
        assert torch.allclose(a.cpu().double(), r, atol=1e-3, rtol=1e-3)
    # and with the fp64 forward's decisions wherever the two agree (away from the kink)
    if code in (0, 2, 3):
        for a, r in ((xg.grad, xr.grad), (Wg.grad, Wr.grad), (bg.grad, br.grad)):
            assert torch.allclose(a.cpu().double(), r, atol=1e-3, rtol=1e-3)


@pytest.mark.gpu
def test_linear_act_backward_without_input_grad(cuda):
    """First layer of a network: no dX; dW / db from the fused weight-gradient kernel alone."""
    from avenir_amd.ops.mlp_ops import linear_act
    g = torch.Generator().manual_seed(4)
    x = torch.randn(5000, 16, generator=g)
    W = torch.randn(48, 16, generator=g) / 4
    b = torch.randn(48, generator=g)
    gy = torch.randn(5000, 48, generator=g)
    Wr, br = W.double().requires_grad_(), b.double().requires_grad_()
    torch.tanh(torch.nn.functional.linear(x.double(), Wr, br)).backward(gy.double())
    Wg, bg = W.to(cuda).requires_grad_(), b.to(cuda).requires_grad_()
    linear_act(x.to(cuda), Wg, bg, "tanh").backward(gy.to(cuda))
    assert torch.allclose(Wg.grad.cpu().double(), Wr.grad, atol=1e-3, rtol=1e-3)
    assert torch.allclose(bg.grad.cpu().double(), br.grad, atol=1e-3, rtol=1e-3)


@pytest.mark.gpu
def test_wgrad_kernel_multi_tile(cuda):
    """The fused weight-gradient binding on a multi-tile layer (N, K > 64, not dispatched by
    linear_act) against float64 torch."""
    from avenir_amd import _native
    g = torch.Generator().manual_seed(6)
    M, K, N = 9000, 130, 96
    x, W = torch.randn(M, K, generator=g), torch.randn(N, K, generator=g) / 10
    y = torch.sigmoid(x @ W.t())
    gy = torch.randn(M, N, generator=g)
    dz = gy.double() * y.double() * (1 - y.double())
    gx, gW, db = _native.C().linear_act_backward(gy.to(cuda), y.to(cuda), x.to(cuda), W.to(cuda), 2, True)
    assert torch.allclose(gW.cpu().double(), dz.t() @ x.double(), atol=2e-3, rtol=1e-3)
    assert torch.allclose(db.cpu().double(), dz.sum(0), atol=2e-3, rtol=1e-3)
    assert torch.allclose(gx.cpu().double(), dz @ W.double(), atol=2e-3, rtol=1e-3)


@pytest.mark.gpu
def test_mlp_fused_trains_on_gpu(cuda):
    x, y = _xor_data()
    m = FeedForwardNetwork("16:relu:false:false:0,16:tanh:false:false:0,2:none:false:false:0", 2, loss="ce",
                           optimizer="adam", lr=0.01, batch_size=64, num_iter=60, device=cuda)
    assert any(type(l).__name__ == "FusedLinear" for l in m.layers)
    m.fit(x, y)
    assert m.evaluate_model(x, y, "accuracy") > 0.95


def test_optimizer_steps_advance_the_param_epoch():
    """Fused optimizers update parameters without bumping their version counters; the packed-weight
    caches also key on the process-wide optimizer-step epoch, which every step advances."""
    from avenir_amd.utils.params import param_epoch
    p = torch.nn.Parameter(torch.randn(5))
    opt = torch.optim.Adam([p], lr=0.1, fused=True)
    p.grad = torch.ones(5)
    e, v = param_epoch(), p._version
    opt.step()
    assert param_epoch() == e + 1
    assert p._version == v          # why the epoch is needed (torch behaviour this guards against)


@pytest.mark.gpu
def test_fused_lstm_with_a_fused_optimizer_matches_foreach(cuda):
    """Eager training of the fused LSTM with torch's fused Adam equals the foreach Adam: the
    packed-weight cache must see fused updates (they leave the version counters alone)."""
    from avenir_amd.ops.rnn import FusedLSTM
    res = []
    for fused in (False, True):
        torch.manual_seed(0)
        m = FusedLSTM(3, 16, 2).to(cuda)
        opt = torch.optim.Adam(m.parameters(), lr=0.05, fused=fused)
        x = torch.randn(32, 5, 3, device=cuda)
        for _ in range(4):
            opt.zero_grad()
            out, _ = m(x)
            out[:, -1].pow(2).sum().backward()
            opt.step()
        res.append({k: v.detach().cpu() for k, v in m.state_dict().items()})
    for k in res[0]:
        assert torch.allclose(res[0][k], res[1][k], atol=1e-5), k
