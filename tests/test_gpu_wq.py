"""GPU parity of the "wq" split-f16 Winograd conv (idf_conv3x3_wq, conv3_wq.hip: each wave owns
all 16 transform positions of its tiles) against fp64 conv2d with the same folded weights --
the wx3 contract (<= 1e-5 scaled, within 4x the exact-f32 kernel's error), plus its scope
(IDF_ERR_UNSUPPORTED outside it), the range guard, batch invariance (the decoder recomputes the
encoder's outputs bit for bit whatever the batch) and idf_conv3x3_wx3 routing to it."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def scaled_err(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).abs() / b.abs().clamp(min=1.0)).max().item()


class Case:
    def __init__(self, B, H, W, C, N, fold=True, scale=1.0, seed=0):
        from idfcodec.packing import round_up, wino_weights, wino_weights_x3
        g = torch.Generator().manual_seed(seed * 1000 + B * 7 + H * 3 + C)
        self.B, self.H, self.W, self.C, self.N = B, H, W, C, N
        self.ld = round_up(C + N, 16) + 4
        self.X = torch.randn(B * H * W, self.ld, generator=g) * scale
        ldw = round_up(C, 16)
        self.n_alloc = round_up(N, 16)
        self.Wt = torch.randn(self.n_alloc, 9, ldw, generator=g, dtype=torch.float64) / np.sqrt(9 * C)
        self.U = wino_weights(self.Wt.numpy(), ldw // 16)
        self.Ux, self.ysc = wino_weights_x3(self.Wt.numpy(), ldw // 16)
        self.b3 = torch.randn(self.n_alloc, generator=g) * 0.1
        self.vt = torch.randn(9, self.n_alloc, generator=g) * 0.1 if fold else None
        self.bfull = None
        if fold:
            s = self.b3.clone()
            for t in range(9):
                s = s + self.vt[t]
            self.bfull = s
        self.fold = fold

    def dev(self):
        d = torch.device("cuda")
        return dict(X=self.X.to(d), U=torch.from_numpy(self.U).to(d),
                    Ux=torch.from_numpy(self.Ux.view(np.int16)).to(d), b3=self.b3.to(d),
                    vt=self.vt.to(d) if self.fold else None,
                    bf=self.bfull.to(d) if self.fold else None)

    def run(self, kind, act="ReLU", check_in=1, X=None, B=None):
        from idfcodec import _lib
        from idfcodec._lib import check, lib, ptr
        B = self.B if B is None else B
        t = self.dev()
        Xd = t["X"] if X is None else X
        H, W, C, N, ld, na = self.H, self.W, self.C, self.N, self.ld, self.n_alloc
        out = torch.zeros(B * H * W, ld, device=Xd.device)
        flag = torch.zeros(1, dtype=torch.int32, device=Xd.device)
        vt, bf = (ptr(t["vt"]), ptr(t["bf"])) if self.fold else (None, None)
        if kind == "wq":
            rc = lib().idf_conv3x3_wq(_lib.stream_ptr(), B, H, W, C, ptr(Xd), ld, ptr(t["Ux"]),
                                      na // 16, self.ysc, ptr(t["b3"]), vt, na, bf, N, ptr(out), ld,
                                      _lib.ACT[act], 0.01, ptr(flag), check_in)
            if rc == 4:  # IDF_ERR_UNSUPPORTED
                return None, None
            check(rc, "wq")
        elif kind == "wx3":
            wsn = lib().idf_conv3x3_wino_workspace(B, H, W, C, N)
            ws = torch.empty(max(wsn, 1), device=Xd.device)
            check(lib().idf_conv3x3_wx3(_lib.stream_ptr(), B, H, W, C, ptr(Xd), ld, ptr(t["Ux"]),
                                        na // 16, self.ysc, ptr(t["b3"]), vt, na, bf, N, ptr(out),
                                        ld, _lib.ACT[act], 0.01, ptr(flag), check_in, ptr(ws), wsn),
                  "wx3")
        else:
            wsn = lib().idf_conv3x3_wino_workspace(B, H, W, C, N)
            ws = torch.empty(max(wsn, 1), device=Xd.device)
            check(lib().idf_conv3x3_wino(_lib.stream_ptr(), B, H, W, C, ptr(Xd), ld, ptr(t["U"]),
                                         na // 16, ptr(t["b3"]), vt, na, bf, N, ptr(out), ld,
                                         _lib.ACT[act], 0.01, ptr(ws), wsn), "wino")
        torch.cuda.synchronize()
        return out.cpu(), int(flag.item())

    def ref(self, act="ReLU"):
        B, H, W, C, N = self.B, self.H, self.W, self.C, self.N
        x4 = self.X[:, :C].double().view(B, H, W, C).permute(0, 3, 1, 2)
        w4 = self.Wt[:N, :, :C].permute(0, 2, 1).reshape(N, C, 3, 3)
        r = F.conv2d(x4, w4, padding=1) + self.b3[:N].double().view(1, -1, 1, 1)
        if self.fold:
            mask = F.conv2d(torch.ones(1, 1, H, W, dtype=torch.float64),
                            torch.eye(9, dtype=torch.float64).view(9, 1, 3, 3), padding=1)
            r = r + torch.einsum("tn,bthw->bnhw", self.vt[:, :N].double(), mask)
        if act == "ReLU":
            return F.relu(r)
        if act == "LeakyReLU":
            return F.leaky_relu(r, 0.01)
        return r

    def err(self, out, act="ReLU"):
        B, H, W, N = self.B, self.H, self.W, self.N
        got = out[:, :N].double().view(B, H, W, N).permute(0, 3, 1, 2)
        assert torch.all(out[:, N:] == 0), "wrote outside the N output columns"
        return scaled_err(got, self.ref(act))


WQ_CASES = [
    (3, 32, 32, 52, 44, "ReLU", True), (5, 16, 16, 100, 44, "ReLU", True),
    (3, 32, 32, 496, 44, "ReLU", True), (1, 16, 16, 520, 44, "ReLU", True),
    (2, 32, 32, 12, 48, "LeakyReLU", True), (1, 45, 37, 20, 44, "ReLU", True),
    (2, 64, 64, 36, 44, "None", False), (3, 16, 16, 200, 96, "ReLU", True),
    (2, 40, 36, 64, 43, "LeakyReLU", True),
]


@pytest.mark.parametrize("B,H,W,C,N,act,fold", WQ_CASES)
def test_wq_vs_fp64(B, H, W, C, N, act, fold):
    c = Case(B, H, W, C, N, fold)
    out, flag = c.run("wq", act)
    assert out is not None, "geometry should be in wq's scope"
    assert flag == 0
    e = c.err(out, act)
    e32 = c.err(c.run("wino", act)[0], act)
    print(f"wq {e:.2e} f32 {e32:.2e}")
    assert e <= 1e-5, f"wq max scaled error {e:.3e}"
    assert e <= max(4 * e32, 1e-6), (e32, e)


@pytest.mark.parametrize("B,H,W,C,N", [(7, 8, 8, 168, 44), (4, 4, 4, 24, 32), (2, 27, 23, 52, 44),
                                       (2, 32, 32, 52, 16)])
def test_wq_out_of_scope(B, H, W, C, N):
    out, _ = Case(B, H, W, C, N).run("wq")
    assert out is None


def test_wx3_routes_to_wq():
    """With IDF_WQ=1 idf_conv3x3_wx3 runs wq where it applies (the same bits as the direct wq
    entry); otherwise it runs its own kernel (other bits, same contract)."""
    import os
    c = Case(2, 32, 32, 100, 44)
    a, _ = c.run("wq")
    b, _ = c.run("wx3")
    if os.environ.get("IDF_WQ") == "1":
        assert torch.equal(a, b)
    else:
        assert c.err(b) <= 1e-5 and c.err(a) <= 1e-5


@pytest.mark.parametrize("H,W", [(32, 32), (16, 16)])
def test_wq_batch_invariant(H, W):
    """An image's outputs do not depend on the batch it is coded in (encoder == decoder)."""
    c = Case(6, H, W, 140, 44, seed=3)
    full, _ = c.run("wq")
    P = H * W
    for i in (0, 3, 5):
        Xi = c.X[i * P:(i + 1) * P].contiguous().cuda()
        one, _ = c.run("wq", X=Xi, B=1)
        assert torch.equal(one, full[i * P:(i + 1) * P]), f"image {i}"


def test_wq_deterministic():
    c = Case(4, 32, 32, 300, 44, seed=5)
    a, _ = c.run("wq")
    b, _ = c.run("wq")
    assert torch.equal(a, b)


def test_wq_range_guard():
    c = Case(2, 32, 32, 52, 44)
    c.X[700, 3] = 40000.0  # |V| >= 32768 on a block input
    out, flag = c.run("wq", check_in=1)
    assert flag == 1
    c2 = Case(2, 32, 32, 52, 44)
    c2.X[100, 0] = float("nan")
    _, flag2 = c2.run("wq", check_in=1)
    assert flag2 == 1
    c3 = Case(2, 16, 16, 52, 44, scale=1e4)  # outputs beyond the output guard
    _, flag3 = c3.run("wq", check_in=0)
    assert flag3 == 1
    _, flag4 = Case(2, 32, 32, 52, 44).run("wq", check_in=1)
    assert flag4 == 0


@pytest.mark.parametrize("scale", [1e-3, 30.0])
def test_wq_far_from_unit_scale(scale):
    c = Case(2, 16, 16, 200, 44, scale=scale)
    out, flag = c.run("wq")
    assert flag == 0
    e, e32 = c.err(out), c.err(c.run("wino")[0])
    assert e <= max(4 * e32, 1e-6), (e32, e)
