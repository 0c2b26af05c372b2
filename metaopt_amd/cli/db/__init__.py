"""``mopt db {setup,test,upgrade}`` (reference: ``cli/db_main.py`` and ``cli/db/``)."""
