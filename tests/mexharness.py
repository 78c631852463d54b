"""ctypes driver of the MEX gateway (matlab/tci_mex.cpp) compiled against the stand-in MATLAB API
(matlab/mexstub/): builds MATLAB values (column-major doubles, logicals, char, struct arrays,
uint64 handles), makes the call ``[out{1:nlhs}] = tci_mex(args{:})`` and reads the results back.
Test infrastructure only."""
from __future__ import annotations

import ctypes as C

import numpy as np

_vp = C.c_void_p


class MexError(Exception):
    """mexErrMsgIdAndTxt inside the gateway: the MATLAB error identifier and message."""

    def __init__(self, ident: str, msg: str):
        super().__init__(f"{ident}: {msg}")
        self.ident = ident
        self.msg = msg


class Mex:
    def __init__(self, path: str):
        L = C.CDLL(path)
        sig = {
            "mxCreateDoubleMatrix": (_vp, [C.c_size_t, C.c_size_t, C.c_int]),
            "mxCreateLogicalMatrix": (_vp, [C.c_size_t, C.c_size_t]),
            "mxCreateString": (_vp, [C.c_char_p]),
            "mxCreateStructMatrix": (_vp, [C.c_size_t, C.c_size_t, C.c_int, C.POINTER(C.c_char_p)]),
            "mxSetField": (None, [_vp, C.c_size_t, C.c_char_p, _vp]),
            "mxDestroyArray": (None, [_vp]),
            "mxGetData": (_vp, [_vp]),
            "mxGetM": (C.c_size_t, [_vp]),
            "mxGetN": (C.c_size_t, [_vp]),
            "mxGetClassID": (C.c_int, [_vp]),
            "mxGetNumberOfDimensions": (C.c_size_t, [_vp]),
            "mxGetDimensions": (C.POINTER(C.c_size_t), [_vp]),
            "mxGetNumberOfFields": (C.c_int, [_vp]),
            "mxGetFieldNameByNumber": (C.c_char_p, [_vp, C.c_int]),
            "mxGetField": (_vp, [_vp, C.c_size_t, C.c_char_p]),
            "mexstub_call": (C.c_int, [C.c_int, C.POINTER(_vp), C.c_int, C.POINTER(_vp)]),
            "mexstub_error_id": (C.c_char_p, []),
            "mexstub_error_msg": (C.c_char_p, []),
            "mexstub_clear": (None, []),
            "mexstub_uint64": (C.c_uint64, [_vp]),
            "mexstub_make_uint64": (_vp, [C.c_uint64]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        self.L = L

    # -- MATLAB values ---------------------------------------------------------------------
    def double(self, a) -> int:
        a = np.asarray(a, np.float64)
        if a.ndim == 0:
            a = a.reshape(1, 1)
        elif a.ndim == 1:
            a = a.reshape(1, -1)  # a MATLAB row vector
        m, n = a.shape
        p = self.L.mxCreateDoubleMatrix(m, n, 0)
        if m * n:
            f = np.asfortranarray(a)   # held until the copy is done (a temporary's buffer would be freed)
            C.memmove(self.L.mxGetData(p), f.ctypes.data, 8 * m * n)
        return p

    def logical(self, a) -> int:
        a = np.asarray(a, bool).reshape(1, -1)
        p = self.L.mxCreateLogicalMatrix(1, a.shape[1])
        if a.size:
            u8 = a.astype(np.uint8)
            C.memmove(self.L.mxGetData(p), u8.ctypes.data, a.size)
        return p

    def string(self, s: str) -> int:
        return self.L.mxCreateString(s.encode())

    def handle(self, v: int) -> int:
        return self.L.mexstub_make_uint64(v)

    def value(self, v) -> int:
        """str -> char, bool -> logical scalar, anything else -> double."""
        if isinstance(v, str):
            return self.string(v)
        if isinstance(v, (bool, np.bool_)):
            return self.logical([bool(v)])
        return self.double(v)

    def struct(self, rows, fields) -> int:
        """A 1 x len(rows) struct array; rows: list of dicts field -> value (numpy, str or bool)."""
        names = (C.c_char_p * len(fields))(*[f.encode() for f in fields])
        p = self.L.mxCreateStructMatrix(1, len(rows), len(fields), names)
        for i, r in enumerate(rows):
            for f in fields:
                if f in r:
                    v = r[f]
                    self.L.mxSetField(p, i, f.encode(), self.value(v))
        return p

    def to_numpy(self, p):
        """A double / uint64 array as numpy (its MATLAB shape, N-D included), a 1x1 struct as a dict."""
        m, n = self.L.mxGetM(p), self.L.mxGetN(p)
        cls = self.L.mxGetClassID(p)
        if cls == 15:  # mxUINT64_CLASS
            return np.array([[self.L.mexstub_uint64(p)]], np.uint64)
        if cls == 2:  # mxSTRUCT_CLASS: field -> value of element 1
            names = [self.L.mxGetFieldNameByNumber(p, f).decode() for f in range(self.L.mxGetNumberOfFields(p))]
            return {f: self.to_numpy(self.L.mxGetField(p, 0, f.encode())) for f in names}
        nd = self.L.mxGetNumberOfDimensions(p)
        dims = tuple(self.L.mxGetDimensions(p)[k] for k in range(nd))
        out = np.empty(m * n, np.float64)
        if m * n:
            C.memmove(out.ctypes.data, self.L.mxGetData(p), 8 * m * n)
        return out.reshape(dims, order="F")  # column-major -> MATLAB's shape

    # -- calls --------------------------------------------------------------------------------
    def call(self, *args, nlhs: int = 1):
        """tci_mex(args...): str -> char, int handle (wrapped by .handle) or a prebuilt mxArray
        pointer; arrays -> double. Returns the nlhs outputs as numpy arrays (inputs are freed)."""
        made = []
        ptrs = []
        for a in args:
            if isinstance(a, MxPtr):
                p = a.p
            elif isinstance(a, str):
                p = self.string(a)
                made.append(p)
            else:
                p = self.double(a)
                made.append(p)
            ptrs.append(p)
        prhs = (_vp * max(len(ptrs), 1))(*ptrs)
        plhs = (_vp * max(nlhs, 1))()
        rc = self.L.mexstub_call(nlhs, plhs, len(ptrs), prhs)
        for p in made:
            self.L.mxDestroyArray(p)
        if rc != 0:
            raise MexError(self.L.mexstub_error_id().decode(), self.L.mexstub_error_msg().decode())
        outs = []
        for i in range(nlhs):
            if plhs[i]:
                outs.append(self.to_numpy(plhs[i]))
                self.L.mxDestroyArray(plhs[i])
            else:
                outs.append(None)
        return outs

    def clear(self):
        """`clear tci_mex`: the gateway's mexAtExit handler (destroys the live contexts)."""
        self.L.mexstub_clear()


class MxPtr:
    """An mxArray built by the caller (kept alive and freed by the caller)."""

    def __init__(self, mex: Mex, p):
        self.mex, self.p = mex, p

    def free(self):
        self.mex.L.mxDestroyArray(self.p)
