"""The command-line tester runs every routine with --check (host target here;
the GPU run exercises target d)."""
import pytest

from slate_d35_amd import tester


def test_tester_all_host(capsys):
    rc = tester.main(["all", "--dim", "150", "--nb", "48", "--type", "d,c", "--target", "h"])
    out = capsys.readouterr().out
    assert rc == 0, out
    assert "all tests passed" in out


@pytest.mark.gpu
def test_tester_all_device(capsys):
    rc = tester.main(["all", "--dim", "300", "--nb", "64", "--type", "d,z", "--target", "d"])
    out = capsys.readouterr().out
    assert rc == 0, out
