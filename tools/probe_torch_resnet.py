"""Probe: plain-PyTorch ResNet-50 v1b training step on one MI355X (MIOpen path).

Used only to size the problem and read the per-kernel breakdown before writing
our own kernels. Not part of the framework.
"""
import sys, time, json
import torch
import torch.nn as nn
import torch.nn.functional as F

class Bottleneck(nn.Module):
    def __init__(self, cin, c, stride, down):
        super().__init__()
        self.c1 = nn.Conv2d(cin, c, 1, bias=False); self.b1 = nn.BatchNorm2d(c)
        self.c2 = nn.Conv2d(c, c, 3, stride, 1, bias=False); self.b2 = nn.BatchNorm2d(c)
        self.c3 = nn.Conv2d(c, c * 4, 1, bias=False); self.b3 = nn.BatchNorm2d(c * 4)
        self.down = None
        if down:
            self.down = nn.Sequential(nn.Conv2d(cin, c * 4, 1, stride, bias=False), nn.BatchNorm2d(c * 4))
    def forward(self, x):
        r = x if self.down is None else self.down(x)
        y = F.relu(self.b1(self.c1(x)))
        y = F.relu(self.b2(self.c2(y)))
        y = self.b3(self.c3(y))
        return F.relu(y + r)

class R50(nn.Module):
    def __init__(self):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(), nn.MaxPool2d(3, 2, 1))
        layers = []; cin = 64
        for i, (n, c) in enumerate([(3, 64), (4, 128), (6, 256), (3, 512)]):
            for j in range(n):
                layers.append(Bottleneck(cin, c, (2 if (j == 0 and i > 0) else 1), j == 0)); cin = c * 4
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(2048, 1000)
    def forward(self, x):
        x = self.layers(self.stem(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))

def run(dtype, bs, steps, warm, cl=True):
    dev = 'cuda'
    m = R50().to(dev)
    if cl: m = m.to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    x = torch.randn(bs, 3, 224, 224, device=dev)
    if cl: x = x.to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (bs,), device=dev)
    def step():
        with torch.autocast('cuda', dtype=dtype):
            loss = F.cross_entropy(m(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
    for _ in range(warm): step()
    torch.cuda.synchronize(); t = time.time()
    for _ in range(steps): step()
    torch.cuda.synchronize(); dt = (time.time() - t) / steps
    return bs / dt, dt * 1000

if __name__ == '__main__':
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    torch.backends.cudnn.benchmark = True
    print(torch.cuda.get_device_name(0), flush=True)
    for dt_name, dt in [('fp16', torch.float16), ('bf16', torch.bfloat16)]:
        ips, ms = run(dt, 256, steps, 5)
        print(json.dumps({'dtype': dt_name, 'img_s': ips, 'ms': ms}), flush=True)
