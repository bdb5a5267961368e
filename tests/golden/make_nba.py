#!/usr/bin/env python3
"""Generate tests/golden/nba.json -- the NBA dataset of the reference's graph tests, as DATA.

Run once in the build container (needs /root/reference and g++):
    python tests/golden/make_nba.py

Source of the data: src/graph/test/TraverseTestBase.h:207-300 (players/teams) and :358-735
(serve/like edges, in insertion order).  Vertex ids are the reference's
``std::hash<std::string>()(name)`` (TraverseTestBase.h:58, :180), computed by compiling a
two-line g++ program so libstdc++'s hash is used exactly.  The expected GO results are the
ones asserted in src/graph/test/GoTest.cpp (line numbers recorded per case); the tag_* cases
keep their $^/$$ tag-prop columns, the older entries of the same queries only their
edge-derived columns.
"""
import json
import re
import subprocess
import tempfile
from pathlib import Path

REF = Path("/root/reference/src/graph/test/TraverseTestBase.h")
OUT = Path(__file__).resolve().parent / "nba.json"


def std_hash(names):
    src = r'''
#include <functional>
#include <iostream>
#include <string>
int main() { std::string s; while (std::getline(std::cin, s)) std::cout << (long long)std::hash<std::string>()(s) << "\n"; }
'''
    with tempfile.TemporaryDirectory() as d:
        c = Path(d) / "h.cpp"
        c.write_text(src)
        exe = Path(d) / "h"
        subprocess.run(["g++", "-O1", "-o", str(exe), str(c)], check=True)
        out = subprocess.run([str(exe)], input="\n".join(names) + "\n", capture_output=True,
                             text=True, check=True).stdout.split()
    return [int(x) for x in out]


def main():
    text = REF.read_text()
    players = re.findall(r'Player\{"([^"]+)",\s*(-?\d+)', text)
    teams = re.findall(r'Team\{"([^"]+)"\}', text)
    serves, likes = [], []
    for m in re.finditer(r'players_\["([^"]+)"\]((?:\s*\.(?:serve|like)\([^)]*\))+)\s*;', text):
        who, chain = m.group(1), m.group(2)
        for call in re.finditer(r'\.(serve|like)\(([^)]*)\)', chain):
            args = [a.strip() for a in call.group(2).split(",")]
            if call.group(1) == "serve":
                serves.append([who, args[0].strip('"'), int(args[1]), int(args[2])])
            else:
                likes.append([who, args[0].strip('"'), int(args[1])])
    names = [p for p, _ in players] + teams + ["NON EXIST VERTEX ID"]
    hashes = std_hash(names)
    vid = dict(zip(names, hashes))
    data = {
        "source": "src/graph/test/TraverseTestBase.h (data), src/graph/test/GoTest.cpp (expectations)",
        "players": [{"name": p, "age": int(a), "vid": vid[p]} for p, a in players],
        "teams": [{"name": t, "vid": vid[t]} for t in teams],
        "serve": serves,     # [player, team, start_year, end_year] in insertion order
        "like": likes,       # [player, other, likeness] in insertion order
        "nonexist_hash": vid["NON EXIST VERTEX ID"],
        # GoTest expectations (values are names; the test maps them to vids)
        "expect": {
            "one_step_serve_tim": {"line": "GoTest.cpp:30-40", "rows": [["Spurs"]]},
            "serve_boris_years": {"line": "GoTest.cpp:41-55",
                                  "rows": [[2003, 2005, "Hawks"], [2005, 2008, "Suns"],
                                           [2008, 2012, "Hornets"], [2012, 2016, "Spurs"],
                                           [2016, 2017, "Jazz"]]},
            "serve_rondo_where": {"line": "GoTest.cpp:56-71",
                                  "rows": [[2014, 2015, "Mavericks"], [2015, 2016, "Kings"],
                                           [2016, 2017, "Bulls"], [2017, 2018, "Pelicans"]]},
            "pipe_boris_like_like_serve": {"line": "GoTest.cpp:72-89",
                                           "rows": [["Spurs"]] * 5 + [["Hornets"], ["Trail Blazers"]]},
            "var_tracy_like_like": {"line": "GoTest.cpp:112-125",
                                    "rows": [["Tracy McGrady"], ["LaMarcus Aldridge"]]},
            "var_pipe_tracy": {"line": "GoTest.cpp:128-143",
                               "rows": [["Kobe Bryant"], ["Grant Hill"], ["Rudy Gay"],
                                        ["Tony Parker"], ["Tim Duncan"]]},
            "distinct_boris_serve_dst": {"line": "GoTest.cpp:213-226 (edge column only)",
                                         "rows": [["Spurs"], ["Hornets"], ["Trail Blazers"]]},
            # cases with $^ / $$ tag props, full rows
            "tag_serve_boris": {"line": "GoTest.cpp:42-56",
                                "rows": [["Boris Diaw", 2003, 2005, "Hawks"],
                                         ["Boris Diaw", 2005, 2008, "Suns"],
                                         ["Boris Diaw", 2008, 2012, "Hornets"],
                                         ["Boris Diaw", 2012, 2016, "Spurs"],
                                         ["Boris Diaw", 2016, 2017, "Jazz"]]},
            "tag_serve_rondo_where": {"line": "GoTest.cpp:57-72",
                                      "rows": [["Rajon Rondo", 2014, 2015, "Mavericks"],
                                               ["Rajon Rondo", 2015, 2016, "Kings"],
                                               ["Rajon Rondo", 2016, 2017, "Bulls"],
                                               ["Rajon Rondo", 2017, 2018, "Pelicans"]]},
            "tag_distinct_nobody": {"line": "GoTest.cpp:221-230", "rows": []},
            "tag_distinct_pipe_dst_team": {"line": "GoTest.cpp:231-246",
                                           "rows": [["Spurs", "Spurs"], ["Hornets", "Hornets"],
                                                    ["Trail Blazers", "Trail Blazers"]]},
            "tag_vertex_not_exist": {"line": "GoTest.cpp:272-289", "rows": []},
            # $-.prop / $var.prop references: input = GO FROM Tim Duncan, Chris Paul
            # OVER like YIELD $^.player.name AS name, like._dst AS id
            "ref_input_yield": {"line": "GoTest.cpp:317-340 (and $var form :364-387)",
                                "rows": [["Tim Duncan", "Manu Ginobili", "Tim Duncan"],
                                         ["Tim Duncan", "Tony Parker", "LaMarcus Aldridge"],
                                         ["Tim Duncan", "Tony Parker", "Manu Ginobili"],
                                         ["Tim Duncan", "Tony Parker", "Tim Duncan"],
                                         ["Chris Paul", "LeBron James", "Ray Allen"],
                                         ["Chris Paul", "Carmelo Anthony", "Chris Paul"],
                                         ["Chris Paul", "Carmelo Anthony", "LeBron James"],
                                         ["Chris Paul", "Carmelo Anthony", "Dwyane Wade"],
                                         ["Chris Paul", "Dwyane Wade", "Chris Paul"],
                                         ["Chris Paul", "Dwyane Wade", "LeBron James"],
                                         ["Chris Paul", "Dwyane Wade", "Carmelo Anthony"]]},
            "ref_input_where": {"line": "GoTest.cpp:341-361 (and $var form :388-407)",
                                "rows": [["Tim Duncan", "Tony Parker", "LaMarcus Aldridge"],
                                         ["Tim Duncan", "Tony Parker", "Manu Ginobili"],
                                         ["Chris Paul", "LeBron James", "Ray Allen"],
                                         ["Chris Paul", "Carmelo Anthony", "LeBron James"],
                                         ["Chris Paul", "Carmelo Anthony", "Dwyane Wade"],
                                         ["Chris Paul", "Dwyane Wade", "LeBron James"],
                                         ["Chris Paul", "Dwyane Wade", "Carmelo Anthony"]]},
            "derived_go3_boris_like": {"line": "derived from the data by P12 (SURVEY 8c)",
                                       "rows": [["Tony Parker"], ["Manu Ginobili"], ["Tim Duncan"],
                                                ["Tony Parker"], ["Tim Duncan"], ["Tim Duncan"],
                                                ["Manu Ginobili"], ["LaMarcus Aldridge"]]},
        },
    }
    OUT.write_text(json.dumps(data, indent=1) + "\n")
    print(f"wrote {OUT}: {len(players)} players, {len(teams)} teams, {len(serves)} serves, {len(likes)} likes")


if __name__ == "__main__":
    main()
