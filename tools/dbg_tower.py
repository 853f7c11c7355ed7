"""Debug harness: one mrec_tower_fwd_bwd call vs a torch emulation of the same
rounding points (prints per-output max errors)."""
import sys
import torch
sys.path.insert(0, ".")
from pytorchrec_amd import dense as D, _mrec

def run(widths, B, seed=0):
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(seed)
    L = len(widths) - 1
    Ws = [(torch.randn(widths[l + 1], widths[l], generator=g) / widths[l] ** 0.5).to(dev) for l in range(L)]
    bs = [(torch.randn(widths[l + 1], generator=g) * 0.1).to(dev) for l in range(L)]
    hw = (torch.randn(widths[-1], generator=g) / widths[-1] ** 0.5).to(dev)
    x0 = torch.zeros(B, D._r8(widths[0]), dtype=torch.bfloat16, device=dev)
    x0[:, :widths[0]] = torch.randn(B, widths[0], generator=g).to(torch.bfloat16).to(dev)
    y = (torch.rand(B, generator=g) < 0.3).float().to(dev)
    imgs = [D.tower_images(W) for W in Ws]
    hs = [D._alloc(B, widths[l + 1], torch.bfloat16, dev) for l in range(L - 1)]
    dhs = [D._alloc(B, widths[l + 1], torch.bfloat16, dev) for l in range(L)]
    dx0 = D._alloc(B, widths[0], torch.bfloat16, dev)
    dz = torch.empty(B, device=dev)
    H = widths[-1]
    npart = int(_mrec.lib().mrec_ctr_head_parts(B))
    ldp = D._r8(H + 1)
    part = torch.empty(npart, ldp, device=dev)
    lp = torch.empty(npart, device=dev)
    loss = torch.empty(1, device=dev)
    a = _mrec.TowerArgs()
    a.batch, a.n_layers = B, L
    for l in range(L + 1):
        a.width[l] = widths[l]
    a.x0, a.ld_x0 = x0.data_ptr(), x0.stride(0)
    for l in range(L):
        a.w_fwd[l], a.w_bwd[l] = imgs[l][0].data_ptr(), imgs[l][1].data_ptr()
        a.bias[l] = bs[l].data_ptr()
        a.dh_out[l], a.ld_dh[l] = dhs[l].data_ptr(), dhs[l].stride(0)
        if l < L - 1:
            a.h_out[l], a.ld_h[l] = hs[l].data_ptr(), hs[l].stride(0)
    a.head_w, a.y = hw.data_ptr(), y.data_ptr()
    a.dx0, a.ld_dx0 = dx0.data_ptr(), dx0.stride(0)
    a.dz, a.part, a.ldp = dz.data_ptr(), part.data_ptr(), ldp
    a.loss_part, a.ticket, a.loss = lp.data_ptr(), D._ticket(dev).data_ptr(), loss.data_ptr()
    _mrec.call("mrec_tower_fwd_bwd", __import__("ctypes").byref(a), _mrec.stream_handle())
    torch.cuda.synchronize()
    # emulation
    rb = lambda t: t.to(torch.bfloat16).float()
    x = x0[:, :widths[0]].float()
    acts = [x]
    for l in range(L):
        x = rb(torch.relu(x @ rb(Ws[l]).T + bs[l]))
        acts.append(x)
    z = acts[-1] @ hw
    d = (torch.sigmoid(z) - y) / B
    print("dz", float((dz - d).abs().max() / d.abs().max()))
    gr = rb(d[:, None] * hw[None, :] * (acts[-1] > 0))
    print("dh_L", float((dhs[-1].float() - gr).abs().max() / gr.abs().max()))
    for l in range(L - 1, -1, -1):
        gx = gr @ rb(Ws[l])
        if l > 0:
            gx = rb(gx * (acts[l] > 0))
            print(f"dh_{l}", float((dhs[l - 1].float() - gx).abs().max() / gx.abs().max()))
        else:
            gx = rb(gx)
            print("dx0", float((dx0.float() - gx).abs().max() / gx.abs().max()))
        gr = gx
    for l in range(L - 1):
        print(f"h_{l+1}", float((hs[l].float() - acts[l + 1]).abs().max() / acts[l + 1].abs().max()))

for w, B in [((100, 512), 16), ((429, 400, 400, 400), 4096), ((45, 70, 33), 1000)]:
    print(w, B)
    run(w, B)

def autograd_paths(widths, B, seed=0):
    from pytorchrec_amd.model.layer import MLP
    dev = torch.device("cuda")
    torch.manual_seed(seed)
    mlp = MLP(widths[0], list(widths[1:]), "relu", 0.0).to(dev)
    head = torch.nn.Linear(widths[-1], 1).to(dev)
    g = torch.Generator().manual_seed(seed)
    x0 = torch.zeros(B, D._r8(widths[0]), dtype=torch.bfloat16, device=dev)
    x0[:, :widths[0]] = torch.randn(B, widths[0], generator=g).to(torch.bfloat16).to(dev)
    x0 = x0[:, :widths[0]]
    y = (torch.rand(B, generator=g) < 0.3).float().to(dev)
    out = []
    for tower in (True, False):
        for p in list(mlp.parameters()) + list(head.parameters()):
            p.grad = None
        xg = x0.detach().requires_grad_()
        if tower:
            loss = D.tower_bce(xg, mlp, head, None, y)
        else:
            loss, _ = D.ctr_head_bce(mlp(xg), head.weight, head.bias, None, y)
        loss.backward()
        out.append([p.grad.clone() for p in mlp.parameters()])
    # torch reference dW0 from emulated dh
    lin = mlp.mlp[0].linear
    rb = lambda t: t.to(torch.bfloat16).float()
    h = rb(torch.relu(x0.float() @ rb(lin.weight).T + lin.bias))
    # single layer only
    z = h @ head.weight.reshape(-1) + head.bias
    d = (torch.sigmoid(z) - y) / B
    dh = rb(d[:, None] * head.weight.reshape(1, -1) * (h > 0))
    dW = dh.T @ x0.float()
    for name, o in zip(("tower", "layered"), out):
        print(name, "dW0 err", float((o[0] - dW).abs().max() / dW.abs().max()),
              "db0 err", float((o[1] - dh.sum(0)).abs().max() / dh.sum(0).abs().max()))

print("autograd (100,512) B=16"); autograd_paths((100, 512), 16)
print("autograd (100,512) B=32"); autograd_paths((100, 512), 32)
print("autograd (100,256) B=16"); autograd_paths((100, 256), 16)
