"""The reference's FPGA communicator (NTT_PCIECommunicationv2.c, built unchanged from its sources
into oracle/_ref by oracle/Makefile) driving lib/terasic_pcie_qsys.so, the Terasic-driver-shaped
shim over libnttmul.  On a GPU box the full transaction must pass the
communicator's own check (NTT_PCIECommunicationv2.c:232-238); without a GPU PCIE_Open fails cleanly."""
import os
import subprocess

import pytest

import nttmul

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "_ref", "ntt_pcie_v2")
SHIM = os.path.join(os.path.dirname(nttmul.LIB_PATH), "terasic_pcie_qsys.so")
needs_exe = pytest.mark.skipif(not os.path.exists(EXE), reason="reference communicator not built")


def _run(tmp_path):
    # PCIE.c:30-33 loads ./terasic_pcie_qsys.so from the cwd; the shim finds libnttmul.so beside
    # itself ($ORIGIN rpath), so a deployment drops both files where the board driver used to be
    os.symlink(SHIM, tmp_path / "terasic_pcie_qsys.so")
    os.symlink(nttmul.LIB_PATH, tmp_path / "libnttmul.so")
    return subprocess.run([EXE], cwd=tmp_path, capture_output=True, text=True, timeout=300)


def test_shim_exports_driver_abi():
    out = subprocess.run(["nm", "-D", "--defined-only", SHIM], capture_output=True, text=True,
                         check=True).stdout
    for sym in ("PCIE_Open", "PCIE_Close", "PCIE_Read32", "PCIE_Write32", "PCIE_Read16",
                "PCIE_Write16", "PCIE_Read8", "PCIE_Write8", "PCIE_DmaWrite", "PCIE_DmaRead",
                "PCIE_DmaFifoWrite", "PCIE_DmaFifoRead"):       # PCIE.c:71-82
        assert f" T {sym}" in out, sym


@needs_exe
@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="GPU present: covered by the gpu test")
def test_reference_communicator_without_gpu(tmp_path):
    r = _run(tmp_path)
    assert "PCIE_Open failed" in r.stdout


@needs_exe
@pytest.mark.gpu
def test_reference_communicator_on_gpu(tmp_path):
    r = _run(tmp_path)
    assert r.returncode == 0, r.stderr
    assert "TB: Sinal 'done_all' recebido!" in r.stdout
    assert "Verificação: 0 erros encontrados." in r.stdout
    assert "Execução NTT falhou" not in r.stdout
