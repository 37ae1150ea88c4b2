"""LstmNetwork data-parallel training: W ranks with local batch b train like one process with
batch W x b (replicas from rank 0, gradients averaged each step) — gloo ranks on the CPU."""
import torch

from tests._dist import run_world


def _data(n=64, T=5, I=2, seed=3):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(n, T * I, generator=g)
    y = (x.sum(1) > T * I / 2).float()
    return x, y


def _net(seed):
    from avenir_amd.nn.sequence import LstmNetwork
    torch.manual_seed(seed)
    return LstmNetwork(2, 8, 1, num_layers=2, seq_len=5, batch_size=1 << 20, lr=0.01, num_iter=3, device="cpu",
                       out_sequence=False)


def _rank_fit(rank, world):
    x, y = _data()
    net = _net(seed=100 + rank)          # different local init: the fit must start from rank 0's
    sh = slice(rank * (64 // world), (rank + 1) * (64 // world))
    net.fit(net.to_sequences(x[sh]), y[sh], num_iter=3)
    return {k: v.detach().clone() for k, v in net.state_dict().items()}, net.losses


def test_two_ranks_equal_one_process_with_the_global_batch():
    x, y = _data()
    ref = _net(seed=100)                 # rank 0's initialisation
    ref.fit(ref.to_sequences(x), y, num_iter=3)
    res = run_world(_rank_fit, 2)
    (sd0, l0), (sd1, l1) = res
    for k, v in ref.state_dict().items():
        assert torch.allclose(sd0[k], v, atol=2e-6, rtol=1e-5), k
        assert torch.equal(sd0[k], sd1[k]), k          # replicas identical
    # the local losses average to the global-batch loss
    for a, b, c in zip(l0, l1, ref.losses):
        assert abs((a + b) / 2 - c) < 1e-5


def _rank_fit_gpu(rank, world):
    import torch as T
    from avenir_amd.nn.sequence import LstmNetwork
    x, y = _data()
    T.manual_seed(100 + rank)
    net = LstmNetwork(2, 8, 1, num_layers=2, seq_len=5, batch_size=1 << 20, lr=0.01, num_iter=3, device="cuda",
                      out_sequence=False)
    sh = slice(rank * (64 // world), (rank + 1) * (64 // world))
    net.fit(net.to_sequences(x[sh]), y[sh], num_iter=3)
    return {k: v.detach().cpu().clone() for k, v in net.state_dict().items()}


import pytest  # noqa: E402


@pytest.mark.gpu
def test_two_ranks_on_the_gpu_equal_one_process(cuda):
    """The fused fp32 LSTM kernels in both ranks (sharing cuda:0, gradients over gloo)."""
    from avenir_amd.nn.sequence import LstmNetwork
    x, y = _data()
    torch.manual_seed(100)
    ref = LstmNetwork(2, 8, 1, num_layers=2, seq_len=5, batch_size=1 << 20, lr=0.01, num_iter=3, device=cuda,
                      out_sequence=False)
    ref.fit(ref.to_sequences(x), y, num_iter=3)
    sd0, sd1 = run_world(_rank_fit_gpu, 2, comm="gloo:cuda")
    for k, v in ref.state_dict().items():
        assert torch.allclose(sd0[k], v.cpu(), atol=1e-5, rtol=1e-4), k
        assert torch.equal(sd0[k], sd1[k]), k


class _DeviceCheckingComm:
    """A 2-rank communicator stand-in that records the device of every tensor the DP fit hands
    it: an RCCL group takes device tensors only (the step-count all-reduce used a host
    tensor, which the library collective rejects)."""
    is_distributed = True
    world, rank = 2, 0

    def __init__(self):
        self.devices = []

    def broadcast(self, t, src=0):
        self.devices.append(t.device.type)
        return t

    def all_reduce(self, t, op="sum", **kw):
        self.devices.append(t.device.type)
        if op == "sum":
            t.mul_(2)
        return t


@pytest.mark.gpu
def test_data_parallel_fit_hands_only_device_tensors_to_the_communicator(cuda):
    from avenir_amd.nn.sequence import LstmNetwork
    x, y = _data()
    net = LstmNetwork(2, 8, 1, num_layers=2, seq_len=5, batch_size=16, lr=0.01, num_iter=1, device="cuda",
                      out_sequence=False)
    net.predict(net.to_sequences(x[:4]))            # builds the packed-weight caches first
    c = _DeviceCheckingComm()
    net.fit(net.to_sequences(x), y, num_iter=1, comm=c)
    assert c.devices and set(c.devices) == {"cuda"}, c.devices
