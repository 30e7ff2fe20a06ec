"""LSMS alloy utilities (reference ``hydragnn/utils/lsms/*``).

* :func:`compute_formation_enthalpy` — binary-alloy formation enthalpy against the
  linear mixing of the two pure-element energies per atom, plus the configurational
  entropy ``k_B ln C(N, N_1)`` in Rydberg/K (``convert_total_energy_to_formation_gibbs.py:130-183``).
* :func:`convert_raw_data_energy_to_gibbs` — rewrite every LSMS file of a directory
  with its formation Gibbs energy ``H_f - T S`` into ``<dir>_gibbs_energy/``.
* :func:`compositional_histogram_cutoff` — keep at most ``histogram_cutoff``
  samples per composition bin (symlinks into ``<dir>_histogram_cutoff/``).

LSMS file layout: line 1 = total energy (Rydberg) [+ other graph values], then one
row per atom whose first column is the element id.
"""
import math
import os
import shutil

import numpy as np

KB_JOULE_PER_KELVIN = 1.380649e-23
JOULE_TO_RYDBERG = 4.5874208973812e17
KB_RYDBERG_PER_KELVIN = KB_JOULE_PER_KELVIN * JOULE_TO_RYDBERG


def _read(path):
    with open(path) as f:
        txt = f.readlines()
    return txt[0].split()[0], txt


def _counts(atoms, elements_list, path=""):
    elements, counts = np.unique(atoms[:, 0], return_counts=True)
    for e in elements:
        assert e in elements_list, f"Sample {path} contains element not present in binary considered."
    full = np.asarray([counts[list(elements).index(e)] if e in elements else 0 for e in elements_list])
    return full


def compute_formation_enthalpy(path, elements_list, pure_elements_energy, total_energy, atoms):
    """-> (composition of element 1, total energy, linear mixing energy, formation enthalpy, entropy)."""
    elements_list = sorted(elements_list)
    counts = _counts(atoms, elements_list, path)
    n = atoms.shape[0]
    comp = counts[0] / n
    mix = (pure_elements_energy[elements_list[0]] * comp + pure_elements_energy[elements_list[1]] * (1 - comp)) * n
    entropy = KB_RYDBERG_PER_KELVIN * math.log(math.comb(int(n), int(counts[0])))
    return comp, total_energy, mix, total_energy - mix, entropy


def convert_raw_data_energy_to_gibbs(dir, elements_list, temperature_kelvin=0, overwrite_data=False,
                                     create_plots=False):
    dir = dir.rstrip("/")
    new_dir = dir + "_gibbs_energy/"
    if os.path.exists(new_dir) and overwrite_data:
        shutil.rmtree(new_dir)
    os.makedirs(new_dir, exist_ok=True)
    elements_list = sorted(elements_list)
    files = sorted(os.listdir(dir))
    pure = {}
    for fn in files:
        e_txt, txt = _read(os.path.join(dir, fn))
        atoms = np.loadtxt(txt[1:], ndmin=2)
        u = np.unique(atoms[:, 0])
        if len(u) == 1:
            pure[u[0]] = float(e_txt) / atoms.shape[0]
    assert len(pure) == 2, "Must have two single element files."
    out = []
    for fn in files:
        path = os.path.join(dir, fn)
        e_txt, txt = _read(path)
        atoms = np.loadtxt(txt[1:], ndmin=2)
        comp, tot, mix, h, s = compute_formation_enthalpy(path, elements_list, pure, float(e_txt), atoms)
        g = h - temperature_kelvin * s
        out.append((comp, tot, mix, h, g))
        txt[0] = txt[0].replace(e_txt, str(g), 1)
        with open(os.path.join(new_dir, fn), "w") as f:
            f.write("".join(txt))
    arr = np.asarray(out)
    print("Min formation enthalpy: ", arr[:, 4].min())
    print("Max formation enthalpy: ", arr[:, 4].max())
    if create_plots:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt

        for k, (x, y, xl, yl, name) in enumerate([
                (1, 2, "Total energy (Rydberg)", "Linear mixing energy (Rydberg)", "linear_mixing_energy.png"),
                (0, 3, "Concentration", "Formation enthalpy (Rydberg)", "formation_enthalpy.png"),
                (0, 4, "Concentration", "Formation Gibbs energy (Rydberg)", "formation_gibbs_energy.png")]):
            plt.figure(k)
            plt.scatter(arr[:, x], arr[:, y], edgecolor="b", facecolor="none")
            plt.xlabel(xl)
            plt.ylabel(yl)
            plt.savefig(name)
    return arr


def find_bin(comp, nbins):
    bins = np.linspace(0, 1, nbins)
    for bi in range(len(bins) - 1):
        if bins[bi] < comp < bins[bi + 1]:
            return bi
    return nbins - 1


def compositional_histogram_cutoff(dir, elements_list, histogram_cutoff, num_bins, overwrite_data=False,
                                   create_plots=False):
    """Down-select LSMS data to at most ``histogram_cutoff`` samples per composition bin."""
    dir = dir.rstrip("/")
    new_dir = dir + "_histogram_cutoff/"
    if os.path.exists(new_dir):
        if not overwrite_data:
            print("Exiting: path to histogram cutoff data already exists")
            return None
        shutil.rmtree(new_dir)
    os.makedirs(new_dir)
    elements_list = sorted(elements_list)
    comp_final, comp_all = [], np.zeros(num_bins)
    for fn in sorted(os.listdir(dir)):
        path = os.path.join(dir, fn)
        atoms = np.loadtxt(path, skiprows=1, ndmin=2)
        counts = _counts(atoms, elements_list, path)
        comp = counts[0] / atoms.shape[0]
        b = find_bin(comp, num_bins)
        comp_all[b] += 1
        if comp_all[b] < histogram_cutoff:
            comp_final.append(comp)
            os.symlink(os.path.abspath(path), os.path.join(new_dir, fn))
    if create_plots:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt

        plt.figure(0)
        plt.hist(comp_final, bins=num_bins)
        plt.savefig("composition_histogram_cutoff.png")
    return comp_final, comp_all
