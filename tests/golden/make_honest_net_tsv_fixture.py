"""Raw text of the data/honest_net.tsv rows the other honest_net fixtures pin (their
`line` numbers), for the TSV writer test (tests/test_csv_runner.py): the header and each
row's fields exactly as the reference's csv_runner wrote them.

    python tests/golden/make_honest_net_tsv_fixture.py /root/reference/data/honest_net.tsv
"""

import json
import pathlib
import sys

HERE = pathlib.Path(__file__).parent


def main(src):
    lines = pathlib.Path(src).read_text().split("\n")
    want = set()
    for name in ("honest_net_clique.json", "honest_net_chains.json"):
        want |= {r["line"] for r in json.loads((HERE / name).read_text())["rows"]}
    out = {"source": "data/honest_net.tsv", "header": lines[0].split("\t"),
           "rows": {str(n): lines[n - 1].split("\t") for n in sorted(want)}}
    (HERE / "honest_net_tsv_lines.json").write_text(json.dumps(out, indent=0))


if __name__ == "__main__":
    main(sys.argv[1])
