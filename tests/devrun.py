"""Device-resident requests for the config-shape GPU tests (test helper).

`DeviceRequest` takes the same (model, data, draws, pars) as hhmm_amd.gqs,
copies the inputs to the GPU once and runs hhmm_run_device on torch's
stream with device-side outputs, so full BASELINE-sized batches (whose
outputs would not fit a host round trip comfortably) can be checked in
place.  Outputs are torch views in the ABI layout, pair fastest:
PTK -> (K, T, P), PT -> (T, P), P -> (P,).
"""
import ctypes as C

import numpy as np
import torch

import hhmm_amd.api
from hhmm_amd import _abi


class DeviceRequest:
    def __init__(self, lib, model, data, draws, pars, pairing="grid", flags=0, uniforms=None, dev=None):
        self.lib = lib
        self.dev = dev or torch.device("cuda", torch.cuda.current_device())
        host = hhmm_amd.api.PreparedRequest(model, data, draws, ["loglik"], pairing)
        req, res = host.req, host.res
        self._keep = {}
        for arr in host.keep:
            self._keep[arr.ctypes.data] = torch.from_numpy(np.asarray(arr).reshape(-1, order="F").copy()).to(
                self.dev)
        for struct in (req.data, req.draws):
            for name, ctype in struct._fields_:
                v = getattr(struct, name)
                if ctype is C.c_void_p and v and v in self._keep:
                    setattr(struct, name, self._keep[v].data_ptr())
        if uniforms is not None:
            uu = np.asarray(uniforms, dtype=np.float64)
            assert uu.shape == (host.P, host.Tmax), uu.shape
            self._keep["ffbs_u"] = torch.from_numpy(uu.reshape(-1, order="F").copy()).to(self.dev)
            req.ffbs_u = self._keep["ffbs_u"].data_ptr()
        P, T, K = host.P, host.Tmax, host.K
        To = host.T_oos_max
        req.outputs = 0
        req.flags = int(flags)
        self.out = {}
        Tz = To if model == "hhmm-tayal2009-lite" else T
        shapes = {"P": (P,), "PTK": (K, T, P), "PT": (T, P), "PTz": (Tz, P), "PToK": (K, To, P)}
        for name in pars:
            dt, code = _abi.RESULT_ARRAYS[name]
            buf = torch.full(shapes[code], float("nan"), dtype=torch.float64, device=self.dev) if dt == "f64" \
                else torch.zeros(shapes[code], dtype=torch.int32, device=self.dev)
            self.out[name] = buf
            req.outputs |= _abi.OUT[name]
            setattr(res, name, buf.data_ptr())
        self.status = torch.zeros(P, dtype=torch.int32, device=self.dev)
        res.pair_status = self.status.data_ptr()
        ws = C.c_size_t(0)
        assert lib.hhmm_workspace_size(C.byref(req), C.byref(ws)) == 0
        self.ws = torch.empty(max(int(ws.value), 256), dtype=torch.uint8, device=self.dev)
        self.req, self.res = req, res
        self.P, self.T, self.K = P, T, K

    def run(self):
        st = self.lib.hhmm_run_device(C.byref(self.req), C.byref(self.res), self.ws.data_ptr(), self.ws.numel(),
                                      torch.cuda.current_stream().cuda_stream)
        if st < 0:
            raise RuntimeError(self.lib.hhmm_last_error().decode())
        torch.cuda.synchronize()
        return st

    def host_pairs(self, name, idx):
        """Outputs of pairs `idx` in gqs()'s host layout ((n, T, K) / (n, T) / (n,))."""
        v = self.out[name]
        ii = torch.as_tensor(np.asarray(idx), device=self.dev)
        if v.dim() == 3:
            return v[:, :, ii].permute(2, 1, 0).cpu().numpy()
        if v.dim() == 2:
            return v[:, ii].T.cpu().numpy()
        return v[ii].cpu().numpy()
