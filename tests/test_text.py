"""Text records (is_text = true): TextRecordExtractor (CP/reader/extractors/raw/TextRecordExtractor.scala:26-108).

CPU: the oracle's literal restatement of the extractor loop against the reference's own text-file
tests (spark-cobol/src/test/.../source/text/Test01AsciiTextFiles.scala:35-60,
Test03AsciiMultisegment.scala:40-120: LF and CRLF files, no trailing line ending) and hand-traced
cases of the window / zero-fill behaviour.  GPU: cbx_frame_text bit-exact against the oracle on
adversarial byte streams (LF, CR, CR LF, lines longer than the window, trailing line endings),
and decoded rows of the reference's text fixtures.
"""
from __future__ import annotations

import numpy as np
import pytest

from oracle import oracle as O
from cobrix_amd import copybook as cbk

T01_COPYBOOK = """       01  RECORD.
           05  A1       PIC X(1).
           05  A2       PIC X(5).
           05  A3       PIC X(10).
"""
T01_TEXT = "\n".join(["1Tes  0123456789", "2 est2 SomeText ", "3None Data¡3    ", "4 on      Data 4"]).encode("utf-8")
T01_EXPECTED = [{"A1": "1", "A2": "Tes", "A3": "0123456789"}, {"A1": "2", "A2": "est2", "A3": "SomeText"},
                {"A1": "3", "A2": "None", "A3": "Data  3"}, {"A1": "4", "A2": "on", "A3": "Data 4"}]

T03_LINES = [b"1Tes  0123456789", b"2Test 01234", b"1None Data  3   ", b"2 on  Data "]


@pytest.mark.parametrize("sep", [b"\n", b"\r\n"])
def test_oracle_reference_multisegment_file(sep):
    data = sep.join(T03_LINES)
    off, ln, vb = O.frame_text(data, 16)
    got = [(data + b"\0" * 32)[o:o + n] for o, n in zip(off, ln)]
    # the last line: its window reached past the data, so it carries the zero fill (ensureBytesRead)
    assert got[:3] == T03_LINES[:3]
    assert got[3] == T03_LINES[3] + b"\0" * (18 - len(T03_LINES[3]))
    assert vb == off[3] + 18


def test_oracle_window_cases():
    # trailing LF after a short last read: one record of zero fill (hasNext: bytesSize > 0)
    off, ln, vb = O.frame_text(b"AB\nCD\n", 3)
    assert list(off) == [0, 3, 6] and list(ln) == [2, 2, 2] and vb == 8
    # no line break: forced records of M - lastFooterSize (1 at the start), then M
    off, ln, vb = O.frame_text(b"X" * 20, 3)
    assert list(off) == [0, 4, 9, 14, 19] and list(ln) == [4, 5, 5, 5, 5] and vb == 24
    # CR at the window's last byte is not a line ending; the LF alone ends the next record
    off, ln, _ = O.frame_text(b"ABCD\r\nEF", 3)   # M = 5
    assert list(off[:2]) == [0, 4] and list(ln[:2]) == [4, 0]
    assert O.frame_text(b"", 3)[0].size == 0
    # a file whose windows end exactly at the data end has no zero fill
    off, ln, vb = O.frame_text(b"ABC\nDE", 4)   # M = 6, one window covers everything
    assert list(off) == [0, 4] and list(ln) == [3, 2] and vb == 6


def _adversarial(rng, n: int) -> bytes:
    alphabet = np.frombuffer(b"\n\r\n\rABCDEFGH  ", dtype=np.uint8)
    parts = []
    total = 0
    while total < n:
        kind = rng.integers(0, 6)
        if kind == 0:
            line = rng.choice(alphabet, size=int(rng.integers(0, 8))).tobytes()
        elif kind == 1:
            line = b"Z" * int(rng.integers(15, 80))   # longer than the window
        else:
            line = bytes(rng.integers(65, 90, size=int(rng.integers(0, 20)), dtype=np.uint8))
        end = [b"\n", b"\r\n", b"\r", b""][int(rng.integers(0, 4))]
        parts.append(line + end)
        total += len(line) + len(end)
    return b"".join(parts)[:n]


@pytest.mark.gpu
class TestGpuText:
    @pytest.fixture(autouse=True)
    def _gpu(self):
        torch = pytest.importorskip("torch")
        if not torch.cuda.is_available():
            pytest.skip("no GPU")
        self.torch = torch

    def _frame(self, data: bytes, record_size: int):
        from cobrix_amd import native as N
        import ctypes
        torch = self.torch
        t = torch.zeros(len(data) + record_size + 64, dtype=torch.uint8, device="cuda")
        if data:
            t[: len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        cap = len(data) + 2
        off = torch.empty(cap, dtype=torch.int64, device="cuda")
        ln = torch.empty(cap, dtype=torch.int32, device="cuda")
        n = ctypes.c_int64(0)
        vb = ctypes.c_int64(0)
        N.check(N.load().cbx_frame_text(t.data_ptr(), len(data), record_size, off.data_ptr(), ln.data_ptr(), cap,
                                        ctypes.byref(n), ctypes.byref(vb),
                                        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
        return off[: n.value].cpu().numpy(), ln[: n.value].cpu().numpy(), vb.value

    @pytest.mark.parametrize("seed,n,rs", [(1, 1, 3), (2, 7, 3), (3, 200, 5), (4, 5000, 16), (5, 100_000, 12),
                                           (6, 777_777, 30), (7, 64, 1)])
    def test_frame_vs_oracle(self, seed, n, rs):
        data = _adversarial(np.random.default_rng(seed), n)
        go, gl, gv = self._frame(data, rs)
        oo, ol, ov = O.frame_text(data, rs)
        assert gv == ov
        np.testing.assert_array_equal(go, oo)
        np.testing.assert_array_equal(gl, ol)

    @pytest.mark.parametrize("data,rs", [(b"", 3), (b"\n", 3), (b"\r\n", 3), (b"\n" * 1000, 2),
                                         (b"X" * 100_003, 7), (b"AB\nCD\n", 3), (b"ABCD\r\nEF", 3),
                                         (b"\r" * 999 + b"\n", 4), ((b"Y" * 21 + b"\r\n") * 3000, 20),
                                         (b"Q" * 50_000 + b"\r\n" + b"R" * 10 + b"\n" + b"S" * 30_001, 5),
                                         ((b"Z" * 700 + b"\n") * 1500, 5), (b"W" * 2_000_001, 3)],
                             ids=["empty", "lf", "crlf", "lf_only", "no_eol", "trailing_lf", "cr_at_window_end",
                                  "cr_run", "crlf_at_window_edge", "few_long_lines", "many_long_lines",
                                  "no_eol_2M"])
    def test_frame_edge_cases(self, data, rs):
        go, gl, gv = self._frame(data, rs)
        oo, ol, ov = O.frame_text(data, rs)
        assert gv == ov
        np.testing.assert_array_equal(go, oo)
        np.testing.assert_array_equal(gl, ol)

    @pytest.mark.parametrize("sep", [b"\n", b"\r\n"])
    def test_all_lines_longer_than_window(self, sep):
        """Every line needs forced records, so every segment's line ending depends on the previous
        one's (bounded walk back; a quadratic walk would time out here)."""
        rng = np.random.default_rng(12)
        lines = [bytes(rng.integers(65, 90, size=int(rng.integers(23, 90)), dtype=np.uint8)) for _ in range(60_000)]
        lines[::97] = [b"\r" * 23] * len(lines[::97])
        data = sep.join(lines)
        go, gl, gv = self._frame(data, 20)
        oo, ol, ov = O.frame_text(data, 20)
        assert gv == ov
        np.testing.assert_array_equal(go, oo)
        np.testing.assert_array_equal(gl, ol)

    @pytest.mark.parametrize("rs,n", [(20, 200_000), (7, 400_000)])
    def test_chained_line_endings(self, rs, n):
        """Lines of 2 * rs + 2 bytes ending in CR LF: every segment's line-ending length depends on
        its predecessor's (a forced record ends right at the CR), so any walk back over segments is
        quadratic here; the map scan is linear."""
        data = (b"Y" * (2 * rs + 2) + b"\r\n") * n
        go, gl, gv = self._frame(data, rs)
        oo, ol, ov = O.frame_text(data, rs)
        assert gv == ov
        np.testing.assert_array_equal(go, oo)
        np.testing.assert_array_equal(gl, ol)

    def test_capacity_reports_required_size(self):
        import ctypes
        from cobrix_amd import native as N
        torch = self.torch
        data = b"AB\nCD\nEF"
        t = torch.zeros(64, dtype=torch.uint8, device="cuda")
        t[: len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        off = torch.empty(8, dtype=torch.int64, device="cuda")
        ln = torch.empty(8, dtype=torch.int32, device="cuda")
        n, vb = ctypes.c_int64(0), ctypes.c_int64(0)
        rc = N.load().cbx_frame_text(t.data_ptr(), len(data), 3, off.data_ptr(), ln.data_ptr(), 1, ctypes.byref(n),
                                     ctypes.byref(vb), None)
        assert rc == N.CBX_E_CAPACITY and n.value >= 2
        rc = N.load().cbx_frame_text(t.data_ptr(), len(data), 3, off.data_ptr(), ln.data_ptr(), 2, ctypes.byref(n),
                                     ctypes.byref(vb), None)
        assert rc == N.CBX_E_CAPACITY and n.value == 3

    def test_reference_ascii_text_file_rows(self):
        from cobrix_amd.reader import ReaderParameters, VarLenNestedReader
        rd = VarLenNestedReader(T01_COPYBOOK, ReaderParameters(is_ebcdic=False, is_text=True,
                                                               schema_policy="collapse_root"))
        assert rd.decode(T01_TEXT).to_rows() == T01_EXPECTED

    @pytest.mark.parametrize("jit", [0, 1])
    def test_text_decode_vs_oracle(self, jit):
        """Text records through the default kernel choice and forced onto the copybook-specialised
        (windowed) kernel the large var-len batches run."""
        from cobrix_amd.reader import ReaderParameters, VarLenNestedReader
        from parity import compare_batch
        data = _adversarial(np.random.default_rng(9), 300_000)
        rd = VarLenNestedReader(T01_COPYBOOK, ReaderParameters(is_ebcdic=False, is_text=True, jit_min_records=jit))
        batch = rd.decode(data)
        off, ln, vb = O.frame_text(data, rd.copybook.record_size)
        padded = data + b"\0" * (vb - len(data))
        errs = compare_batch(batch, O.decode_var(rd.copybook, padded, off, ln))
        assert not errs, errs
