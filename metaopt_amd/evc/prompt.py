"""Interactive branching-conflict resolver, a ``cmd.Cmd`` REPL
(reference: ``src/orion/core/io/interactive_commands/branching_prompt.py:77-485``).

Commands: ``status``, ``diff``, ``auto``, ``name``, ``code``, ``commandline``, ``config``,
``algo``, ``add``, ``remove``, ``rename``, ``reset``, ``commit``, ``abort``, ``quit``/``q``,
``shell``/``!``, ``help``/``h``.  Only started on a TTY; tests drive it with ``onecmd``.
"""
from __future__ import annotations

import cmd
import io
import shlex
import subprocess

from ..space.dims import Dimension
from . import adapters
from . import conflicts as C

GREEN, RED, END = "\033[32m", "\033[31m", "\033[0m"


def _green(s):
    return f"{GREEN}{s}{END}"


def _red(s):
    return f"{RED}{s}{END}"


class BranchingPrompt(cmd.Cmd):
    intro = ("\n\nWelcome to the experiment branching interactive conflicts resolver\n"
             "-----------------------------------------------------------------\n\n"
             "Type `help` to print the help message, `abort` or `(q)uit` to quit without saving.\n"
             "\n%s")
    prompt = "(mopt) "

    def __init__(self, branch_builder, stdin=None, stdout=None):
        super().__init__(stdin=stdin, stdout=stdout)
        if stdin is not None:
            self.use_rawinput = False
        self.branch_builder = branch_builder
        self.abort = False

    def _print(self, *args):
        print(*args, file=self.stdout)

    def cmdloop(self, intro=None):
        super().cmdloop(self.intro % self.get_status())

    def solve_conflicts(self):
        self.cmdloop()

    def get_status(self, options=None) -> str:
        out = io.StringIO()
        conflicts = self.branch_builder.conflicts
        resolved, remaining = conflicts.get_resolved(), conflicts.get_remaining()
        if resolved:
            print("Resolutions:\n", file=out)
            for r in sorted(set(str(c.resolution) for c in resolved if c.resolution is not None)):
                print("    ", _green(r), file=out)
            print(file=out)
        if remaining:
            print("Remaining conflicts:\n", file=out)
            for c in remaining:
                print("    ", _red(repr(c)), file=out)
            print(file=out)
        if not resolved and not remaining:
            print("No conflicts", file=out)
        return out.getvalue()

    # -- commands -----------------------------------------------------------------------------
    def do_status(self, arg):
        """Display the current status of the conflicting configuration."""
        self._print(self.get_status())

    def do_diff(self, arg):
        """Print the diff of every conflict still unresolved."""
        for c in self.branch_builder.conflicts.get_remaining():
            d = c.diff
            if d:
                self._print(repr(c))
                self._print(d)
                self._print()

    def do_auto(self, arg):
        """Automatically resolve every conflict that can be resolved with default choices."""
        conflicts = self.branch_builder.conflicts
        for c in conflicts.get_remaining():
            conflicts.try_resolve(c, silence_errors=True)
        self._print(self.get_status())

    def do_name(self, arg):
        """name <experiment-name>: branch to a new experiment name."""
        self._safe(self.branch_builder.change_experiment_name, arg.strip())

    def do_code(self, arg):
        """code {noeffect,break,unsure}: set the type of code change."""
        self._change_type(arg, adapters.CodeChange, self.branch_builder.set_code_change_type)

    def do_commandline(self, arg):
        """commandline {noeffect,break,unsure}: set the type of command line change."""
        self._change_type(arg, adapters.CommandLineChange, self.branch_builder.set_cli_change_type)

    def do_config(self, arg):
        """config {noeffect,break,unsure}: set the type of script configuration change."""
        self._change_type(arg, adapters.ScriptConfigChange,
                          self.branch_builder.set_script_config_change_type)

    def do_algo(self, arg):
        """Resolve the algorithm configuration conflict."""
        self._safe(self.branch_builder.set_algo)

    def do_add(self, arg):
        """add <dimension> [--default-value V]: add a new or changed dimension."""
        name, default = self._name_default(arg)
        self._safe(self.branch_builder.add_dimension, name, default)

    def do_remove(self, arg):
        """remove <dimension> [--default-value V]: remove a missing dimension."""
        name, default = self._name_default(arg)
        self._safe(self.branch_builder.remove_dimension, name, default)

    def do_rename(self, arg):
        """rename <old-name> <new-name>: rename a missing dimension to a new one."""
        parts = shlex.split(arg)
        if len(parts) != 2:
            self._print("usage: rename <old-name> <new-name>")
            return
        self._safe(self.branch_builder.rename_dimension, parts[0], parts[1])

    def do_reset(self, arg):
        """reset '<resolution>' ...: revert resolutions (as printed by `status`)."""
        for res in shlex.split(arg):
            self._safe(self.branch_builder.reset, res)

    def do_commit(self, arg):
        """Commit the resolutions and exit (only when every conflict is resolved)."""
        if not self.branch_builder.is_resolved:
            self._print("There are still conflicts to solve:")
            self._print(self.get_status())
            return False
        return True

    def do_abort(self, arg):
        """Exit without saving the resolutions."""
        self.abort = True
        return True

    def do_quit(self, arg):
        """Exit without saving the resolutions."""
        return self.do_abort(arg)

    do_q = do_quit

    def do_shell(self, arg):
        """Run a shell command (also `!command`)."""
        proc = subprocess.run(arg, shell=True, capture_output=True, text=True)
        self._print(proc.stdout + proc.stderr)

    def do_h(self, arg):
        """Alias of help."""
        return self.do_help(arg)

    def do_EOF(self, arg):  # noqa: N802 - cmd's name for end of input
        self.abort = True
        return True

    # -- helpers ------------------------------------------------------------------------------
    def _safe(self, fn, *args):
        try:
            fn(*args)
        except (ValueError, RuntimeError, IndexError) as exc:
            self._print(f"Invalid: {exc}")

    def _change_type(self, arg, adapter_cls, setter):
        t = arg.strip()
        if t not in adapter_cls.types:
            self._print(f"Invalid change type '{t}'; choose one of {adapter_cls.types}")
            return
        self._safe(setter, t)

    @staticmethod
    def _name_default(arg):
        parts = shlex.split(arg)
        name = parts[0] if parts else ""
        default = Dimension.NO_DEFAULT_VALUE
        if "--default-value" in parts:
            i = parts.index("--default-value")
            if i + 1 < len(parts):
                default = parts[i + 1]
        return name, default

    def complete_add(self, text, line, begidx, endidx):
        return self._complete_dims(text, [C.NewDimensionConflict, C.ChangedDimensionConflict])

    def complete_remove(self, text, line, begidx, endidx):
        return self._complete_dims(text, [C.MissingDimensionConflict])

    def complete_rename(self, text, line, begidx, endidx):
        return self._complete_dims(text, [C.MissingDimensionConflict, C.NewDimensionConflict])

    def _complete_dims(self, text, types):
        from ..utils.format_trials import standard_param_name
        names = [standard_param_name(c.dimension.name)
                 for c in self.branch_builder.conflicts.get_remaining(types)]
        return [n for n in names if n.startswith(text)]
