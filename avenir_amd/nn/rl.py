"""Deep Q-learning for dynamic pricing on a vectorised device environment.

Reference: ``HiLoPricingEnv`` + Ray RLlib DQN (P/app/price_rl.py:40-265: T=20 price steps, price grid
400..495 step 5, demand = intercept + k1*dp + k2*dp^2 - a*sqrt(increase) + b*sqrt(decrease) +
cyclic term + N(0, 100) noise, reward = demand * (price - unit cost); DQN lr 0.002, gamma 0.8,
train batch 256, hiddens [128, 128, 128], checkpoint / restore / incremental training), plus the
policy server/client pair (price_rl_srv.py / price_rl_clnt.py).

MI355X design: instead of one Python gym environment stepped per transition, ``E`` pricing
environments advance together as device tensors ([E, 2T+1] state), the replay buffer is a device
ring of transitions, and each training step is one batched Double-DQN update — no Ray, no host
round trips inside an episode.  ``PolicyServer`` exposes greedy actions for external clients.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from .common import load_checkpoint, pick_device, save_checkpoint


@dataclass
class PricingParams:
    T: int = 20
    price_min: float = 400
    price_max: float = 500
    price_step: float = 5
    intercept: float = 5000
    k1: float = -5.0
    k2: float = -0.1
    unit_cost: float = 100
    a_inc: float = 300
    b_dec: float = 100
    cyc_amp: float = 500
    rand_sd: float = 100

    @property
    def grid(self):
        return torch.arange(self.price_min, self.price_max, self.price_step)

    @property
    def cyc_period(self):
        return 5 * self.T

    @property
    def state_size(self):
        return 2 * self.T + 1


class PricingEnv:
    """E environments at once; state = [past T prices | one-hot time step | cycle offset]."""

    def __init__(self, n_envs: int, params: PricingParams | None = None, device=None, seed: int = 0):
        self.p = params or PricingParams()
        self.E = n_envs
        self.device = pick_device(device)
        self.g = torch.Generator(device=self.device).manual_seed(seed)
        self.grid = self.p.grid.to(self.device).float()
        self.n_actions = self.grid.numel()
        self.reset()

    def reset(self) -> torch.Tensor:
        p = self.p
        self.state = torch.zeros((self.E, p.state_size), device=self.device)
        self.state[:, -1] = torch.randint(0, p.cyc_period + 1, (self.E,), device=self.device, generator=self.g).float()
        self.t = 0
        return self.state.clone()

    def demand(self, cur, prev, coff):
        p = self.p
        pdm = cur - p.price_min
        pdp = cur - prev
        q = p.intercept + p.k1 * pdm + p.k2 * pdm * pdm - p.a_inc * pdp.clamp_min(0).sqrt() \
            + p.b_dec * (-pdp).clamp_min(0).sqrt()
        q = q + p.cyc_amp * torch.sin(2 * math.pi * coff / p.cyc_period)
        q = q + p.rand_sd * torch.randn(cur.shape, device=self.device, generator=self.g)
        return q.clamp_min(0)

    def step(self, action: torch.Tensor):
        p, T = self.p, self.p.T
        nxt = torch.zeros_like(self.state)
        nxt[:, 0] = self.grid[action]
        nxt[:, 1:T] = self.state[:, 0:T - 1]
        nxt[:, T + self.t] = 1
        nxt[:, -1] = (self.state[:, -1] + 1) % p.cyc_period
        reward = self.demand(nxt[:, 0], nxt[:, 1], nxt[:, -1]) * (nxt[:, 0] - p.unit_cost)
        self.t += 1
        self.state = nxt
        done = self.t == T - 1
        return nxt.clone(), reward, done


class QNetwork(torch.nn.Module):
    """Hidden layers as the framework's fused Linear + ReLU (nn/mlp.py ``FusedLinear`` -> the K27
    kernel of mlp.hip on the GPU, forward and backward); ``fused=False`` builds the plain
    ``torch.nn`` twin with the same parameter names (``net.<2i>.weight``)."""

    def __init__(self, n_in: int, n_actions: int, hiddens=(128, 128, 128), fused: bool = True):
        super().__init__()
        from .mlp import FusedLinear
        layers, d = [], n_in
        for h in hiddens:
            if fused:
                layers += [FusedLinear(d, h, "relu"), torch.nn.Identity()]
            else:
                layers += [torch.nn.Linear(d, h), torch.nn.ReLU()]
            d = h
        layers.append(FusedLinear(d, n_actions, "none") if fused else torch.nn.Linear(d, n_actions))
        self.net = torch.nn.Sequential(*layers)

    def forward(self, x):
        return self.net(x)


class DQNAgent:
    """Double DQN with a device replay ring and a periodically synced target network.

    On the GPU one ``learn`` — replay sampling, the double-DQN target, the Huber loss, backward,
    fused Adam and the target-network sync — is ONE captured HIP graph (``graph=True``): the
    replay size and the update counter live on the device, the sampling draws from the agent's
    generator (registered with the graph, so replays continue its Philox stream exactly as eager
    calls would) and the sync is a masked ``lerp`` (weight 1 every ``target_sync`` updates, else
    0) instead of a host branch.  ``fused=False`` / ``graph=False`` give the eager ``torch.nn``
    twin used by the equivalence tests."""

    def __init__(self, env: PricingEnv, lr: float = 0.002, gamma: float = 0.8, batch: int = 256,
                 hiddens=(128, 128, 128), buffer: int = 100_000, eps_start: float = 1.0, eps_end: float = 0.05,
                 eps_decay_steps: int = 2000, target_sync: int = 200, reward_scale: float = 1e-6, seed: int = 0,
                 fused: bool = True, graph: bool = True):
        self.env = env
        dev = env.device
        self.device = dev
        S, A = env.p.state_size, env.n_actions
        self.scale = torch.tensor([1.0 / env.p.price_max] * env.p.T + [1.0] * env.p.T + [1.0 / env.p.cyc_period],
                                  device=dev)
        self.q = QNetwork(S, A, hiddens, fused=fused).to(dev)
        self.q_tgt = QNetwork(S, A, hiddens, fused=fused).to(dev)
        self.q_tgt.load_state_dict(self.q.state_dict())
        cuda = dev.type == "cuda"
        # fused single-kernel Adam, capturable (its step counter on the device) on the GPU
        self.opt = torch.optim.Adam(self.q.parameters(), lr=lr, fused=True if cuda else None, capturable=cuda)
        self.use_graph = bool(graph and cuda)
        self._graph = None
        self._gloss = None
        self._size_dev = torch.zeros((), device=dev)              # replay fill level (float, for sampling)
        self._steps_dev = torch.zeros((), dtype=torch.long, device=dev)
        self.gamma, self.batch, self.reward_scale = gamma, batch, reward_scale
        self.cap = buffer
        self.buf_s = torch.zeros((buffer, S), device=dev)
        self.buf_a = torch.zeros((buffer,), dtype=torch.long, device=dev)
        self.buf_r = torch.zeros((buffer,), device=dev)
        self.buf_s2 = torch.zeros((buffer, S), device=dev)
        self.buf_d = torch.zeros((buffer,), device=dev)
        self.ptr = 0
        self.size = 0
        self.steps = 0
        self.eps_start, self.eps_end, self.eps_decay = eps_start, eps_end, eps_decay_steps
        self.target_sync = target_sync
        self.g = torch.Generator(device=dev).manual_seed(seed)
        self.episode_rewards: list[float] = []

    def epsilon(self):
        f = min(1.0, self.steps / max(self.eps_decay, 1))
        return self.eps_start + f * (self.eps_end - self.eps_start)

    @torch.no_grad()
    def act(self, s: torch.Tensor, greedy: bool = False) -> torch.Tensor:
        qa = self.q(s * self.scale).argmax(1)
        if greedy:
            return qa
        rnd = torch.randint(0, self.env.n_actions, qa.shape, device=self.device, generator=self.g)
        explore = torch.rand(qa.shape, device=self.device, generator=self.g) < self.epsilon()
        return torch.where(explore, rnd, qa)

    def _store(self, s, a, r, s2, d):
        n = s.shape[0]
        idx = (torch.arange(n, device=self.device) + self.ptr) % self.cap
        self.buf_s[idx], self.buf_a[idx], self.buf_r[idx], self.buf_s2[idx] = s, a, r, s2
        self.buf_d[idx] = float(d)
        self.ptr = (self.ptr + n) % self.cap
        self.size = min(self.size + n, self.cap)
        self._size_dev.fill_(float(self.size))        # a fill kernel: no host synchronisation

    def _learn_body(self) -> torch.Tensor:
        """One Double-DQN update; device-only (capturable)."""
        u = torch.rand((self.batch,), device=self.device, generator=self.g)
        i = (u * self._size_dev).long().clamp_max(self.cap - 1)
        s, a, r, s2, d = self.buf_s[i] * self.scale, self.buf_a[i], self.buf_r[i] * self.reward_scale, \
            self.buf_s2[i] * self.scale, self.buf_d[i]
        with torch.no_grad():
            a2 = self.q(s2).argmax(1, keepdim=True)
            tgt = r + self.gamma * (1 - d) * self.q_tgt(s2).gather(1, a2).squeeze(1)
        q = self.q(s).gather(1, a.view(-1, 1)).squeeze(1)
        loss = torch.nn.functional.smooth_l1_loss(q, tgt)
        self.opt.zero_grad(set_to_none=False)
        loss.backward()
        self.opt.step()
        with torch.no_grad():
            self._steps_dev += 1
            m = (self._steps_dev % self.target_sync == 0).to(torch.float32)
            for t, p in zip(self.q_tgt.parameters(), self.q.parameters()):
                t.lerp_(p, m)                             # target sync: weight 1 every target_sync updates
        return loss.detach()

    def _capture(self):
        """Warm up (allocator pools, Adam state) on a side stream, restore every piece of state the
        warm-up touched, then capture one update."""
        from ..utils.hipgraph import capturing
        ps = [t for m in (self.q, self.q_tgt) for t in m.parameters()]
        snap = [t.detach().clone() for t in ps]
        ost = {id(p): {k: v.clone() for k, v in st.items() if torch.is_tensor(v)} for p, st in self.opt.state.items()}
        gst, steps0 = self.g.get_state(), self._steps_dev.clone()
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(3):
                self._learn_body()
        torch.cuda.current_stream(self.device).wait_stream(side)
        with torch.no_grad():
            for t, v in zip(ps, snap):
                t.copy_(v)
            for p, st in self.opt.state.items():   # restored moments (restore()) or a fresh state
                old = ost.get(id(p), {})
                for k, v in st.items():
                    if torch.is_tensor(v):
                        v.copy_(old[k]) if k in old else v.zero_()
            self._steps_dev.copy_(steps0)
        self.g.set_state(gst)
        self._graph = torch.cuda.CUDAGraph()
        self._graph.register_generator_state(self.g)
        with capturing(self._graph, device=self.device):
            self._gloss = self._learn_body()

    def learn(self):
        if self.size < self.batch:
            return None
        if self.use_graph:
            if self._graph is None:
                self._capture()
            self._graph.replay()
            loss = self._gloss
        else:
            loss = self._learn_body()
        self.steps += 1
        return loss

    def train(self, iterations: int = 50, updates_per_step: int = 1):
        """One iteration = one episode of all E environments (T-1 steps)."""
        for _ in range(iterations):
            s = self.env.reset()
            total = torch.zeros(self.env.E, device=self.device)
            done = False
            while not done:
                a = self.act(s)
                s2, r, done = self.env.step(a)
                self._store(s, a, r, s2, done)
                total += r
                for _ in range(updates_per_step):
                    self.learn()
                s = s2
            self.episode_rewards.append(float(total.mean()))
        return self

    @torch.no_grad()
    def evaluate(self, episodes: int = 1) -> float:
        tot = 0.0
        for _ in range(episodes):
            s = self.env.reset()
            done = False
            ep = torch.zeros(self.env.E, device=self.device)
            while not done:
                s, r, done = self.env.step(self.act(s, greedy=True))
                ep += r
            tot += float(ep.mean())
        return tot / episodes

    def save(self, path):
        save_checkpoint(path, self.q, self.opt, steps=self.steps)

    def restore(self, path):
        st = load_checkpoint(path, self.q, self.opt)
        self.q_tgt.load_state_dict(self.q.state_dict())
        self.steps = int(st.get("steps", 0))
        self._steps_dev.fill_(self.steps)
        self._graph = None                   # re-capture: the optimiser state tensors were replaced


class PolicyServer:
    """In-process policy endpoint (price_rl_srv.py): ``get_action(state)`` returns greedy prices;
    ``log_returns`` accumulates rewards reported by clients for incremental training."""

    def __init__(self, agent: DQNAgent):
        self.agent = agent
        self.returns: list[float] = []

    def get_action(self, state) -> list[int]:
        s = torch.as_tensor(state, dtype=torch.float32, device=self.agent.device).view(-1, self.agent.env.p.state_size)
        return self.agent.act(s, greedy=True).tolist()

    def get_price(self, state) -> list[float]:
        return [float(self.agent.env.grid[a]) for a in self.get_action(state)]

    def log_returns(self, reward: float):
        self.returns.append(float(reward))
