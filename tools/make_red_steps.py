#!/usr/bin/env python3
"""Stage the reference's scripted red action profiles (red_steps.csv,
red_steps2.csv, red_steps3.csv: 40 rows of [radar, salvo, course, speed] read
by Game.define_red_actions, game.py:173-182) as package data
lnw/data/red_steps.npy, float64 [3, 40, 4]. Run in the container that holds
/root/reference; the GPU box uses the committed .npy."""
import csv
import os

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "littoral-naval-warfare-marl_amd", "lnw", "data", "red_steps.npy")
tabs = []
for f in ("red_steps.csv", "red_steps2.csv", "red_steps3.csv"):
    with open(os.path.join(REF, f)) as fh:
        tabs.append([[float(c) for c in row] for row in csv.reader(fh)])
np.save(OUT, np.array(tabs, np.float64))
print(OUT, np.array(tabs).shape)
