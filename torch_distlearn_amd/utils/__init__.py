from .walk import walk_table, walkTable, map_table, clone_table
from .color_print import printServer, printClient, set_verbose
