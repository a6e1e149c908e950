"""acados_template.plot_utils.latexify_plot (imported by the reference's store_results.py:5).
Sets matplotlib's text/font parameters when matplotlib is present; otherwise a no-op."""


def latexify_plot(fontsize=12):
    try:
        import matplotlib
    except ImportError:
        return
    matplotlib.rcParams.update({"axes.labelsize": fontsize, "axes.titlesize": fontsize,
                                "legend.fontsize": fontsize, "xtick.labelsize": fontsize,
                                "ytick.labelsize": fontsize, "font.family": "serif"})
