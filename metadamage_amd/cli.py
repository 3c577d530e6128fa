"""`metadamage` command line (mirror of /root/reference/metadamage/cli.py).

Same sub-command and flags as the reference's `metadamage fit` (cli.py:97-159)
so existing invocations keep working; `--version` as cli.py:72-77.  The
`dashboard` sub-command is out of scope (the reference's Dash viewer reads the
parquet files this writes unchanged); it reports that and exits non-zero.
"""

from __future__ import annotations

import logging
from pathlib import Path
from typing import List, Optional

import typer

from . import utils
from .__version__ import __version__
from .main import main

out_dir_default = Path("./data/out/")

cli_app = typer.Typer(add_completion=False)


def version_callback(value: bool):
    if value:
        typer.echo(f"Metadamage CLI, version: {__version__}")
        raise typer.Exit()


@cli_app.callback()
def callback(version: Optional[bool] = typer.Option(None, "--version", callback=version_callback)):
    """
    Metagenomics Ancient Damage: metadamage (MI355X engine).

    Run the fit command:

    \b
        $ metadamage fit --help
    """


@cli_app.command("fit")
def cli_fit(
    filenames: List[Path] = typer.Argument(...),
    out_dir: Path = typer.Option(out_dir_default),
    max_fits: Optional[int] = typer.Option(None, help="[default: None (All fits)]"),
    max_cores: int = 1,
    min_alignments: int = 10,
    min_y_sum: int = 10,
    substitution_bases_forward: utils.SubstitutionBases = typer.Option(utils.SubstitutionBases.CT),
    substitution_bases_reverse: utils.SubstitutionBases = typer.Option(utils.SubstitutionBases.GA),
    forced: bool = typer.Option(False, "--forced"),
    inference: str = typer.Option("nuts", help="nuts: NUTS sampling as the reference; map: MAP fit"),
):
    """Fitting Ancient Damage.

    FILENAME is the name of the file(s) to fit (with the ancient-model)

    \b
        $ metadamage fit --max-fits 10 --max-cores 2 ./data/input/data_ancient.txt
    """
    logging.basicConfig(level=logging.WARNING, format="%(message)s")
    d_cfg = {
        "out_dir": out_dir,
        "max_fits": max_fits,
        "max_cores": max_cores,
        "min_alignments": min_alignments,
        "min_y_sum": min_y_sum,
        "substitution_bases_forward": substitution_bases_forward.value,
        "substitution_bases_reverse": substitution_bases_reverse.value,
        "forced": forced,
        "version": "0.0.0",
        "inference": inference,
    }
    if inference not in ("nuts", "map"):
        raise typer.BadParameter("--inference must be nuts or map")
    cfg = utils.Config(**d_cfg)
    cfg.add_filenames(filenames)
    # launched by torchrun (WORLD_SIZE > 1): one rank per GPU, the rank's GPU
    # selected before any device call, RCCL process group; main() then deals
    # files or shards taxa over the ranks and rank 0 writes the shared results
    from .distributed import run_distributed

    run_distributed(main, filenames, cfg)


@cli_app.command("dashboard")
def cli_dashboard(dir: Path = typer.Argument(out_dir_default), debug: bool = typer.Option(False, "--debug")):
    """Dashboard: not part of this engine (the reference dashboard reads its output as-is)."""
    typer.echo("The dashboard is not part of metadamage_amd; run the reference `metadamage dashboard "
               f"{dir}` on the output directory.")
    raise typer.Exit(code=2)


def cli_main():
    cli_app(prog_name="metadamage")
