import torch, sys
sys.path.insert(0, '.')
from avenir_amd.ops import rnn
torch.manual_seed(37)
for (B,T,I,H) in [(37,5,3,20),(64,5,3,20),(37,1,3,20),(37,5,3,32),(16,3,3,32)]:
    k = 1.0 / H ** 0.5
    x = torch.randn(B, T, I, device='cuda')
    w_ih = (torch.rand(4 * H, I, device='cuda') * 2 - 1) * k
    w_hh = (torch.rand(4 * H, H, device='cuda') * 2 - 1) * k
    b = (torch.rand(4 * H, device='cuda') * 2 - 1) * k
    for use_h0 in (False, True):
        h0 = torch.randn(B, H, device='cuda') * 0.5 if use_h0 else None
        c0 = torch.randn(B, H, device='cuda') * 0.5 if use_h0 else None
        with torch.no_grad():
            hs, h, c = rnn.lstm_layer(x, w_ih, w_hh, b, h0, c0)
            hr, (h_r, c_r) = rnn.lstm_reference(x.double(), w_ih.double(), w_hh.double(), b.double(),
                                                None if h0 is None else h0.double(), None if c0 is None else c0.double())
        e = (hs.double() - hr).abs()
        print(B,T,I,H,'h0' if use_h0 else '--', 'max', e.max().item(), 'per t', [round(v,4) for v in e.amax(dim=(0,2)).tolist()],
              'worst unit', e.amax(dim=(0,1)).argmax().item(), 'worst row', e.amax(dim=(1,2)).argmax().item())
