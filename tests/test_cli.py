"""The reference's own CLI tests (/root/reference/tests/test_metadamage.py),
run against this package's `metadamage` app."""

from pathlib import Path

from typer.testing import CliRunner

from metadamage_amd.cli import cli_app
from metadamage_amd.utils import extract_name


def test_extracting_name_from_string():
    assert extract_name("./data/input/data_ancient.txt") == "data_ancient"


def test_extracting_name_from_path():
    assert extract_name(Path("./data/input/data_ancient.txt")) == "data_ancient"


def test_cli_fit_bad_file():
    result = CliRunner().invoke(cli_app, ["fit", "file_which_does_not_exist.txt"])
    assert result.exit_code == 1
    assert isinstance(result.exception, Exception)


def test_cli_fit_bad_files():
    result = CliRunner().invoke(
        cli_app, ["fit", "file_which_does_not_exist.txt", "another_file_which_does_not_exist.txt"])
    assert result.exit_code == 1
    assert isinstance(result.exception, Exception)


def test_cli_fit_version():
    result = CliRunner().invoke(cli_app, ["--version"])
    assert result.exit_code == 0
    assert "version" in result.stdout


def test_cli_fit_flags_match_reference():
    """Every flag of the reference's `metadamage fit` (cli.py:97-121) exists."""
    import typer

    cmd = typer.main.get_command(cli_app).commands["fit"]
    opts = {o for p in cmd.params for o in getattr(p, "opts", [])}
    for flag in ("--out-dir", "--max-fits", "--max-cores", "--min-alignments", "--min-y-sum",
                 "--substitution-bases-forward", "--substitution-bases-reverse", "--forced"):
        assert flag in opts, flag
