"""Device memory management: workspaces (MemoryWorkspace arenas, SCOPE_PANIC) sized for 288 GB HBM per GPU."""
from .workspace import (AllocationPolicy, LearningPolicy, LocationPolicy, MemoryWorkspace, MirroringPolicy,
                        ND4JWorkspaceException, ResetPolicy, SpillPolicy, WorkspaceConfiguration, WorkspaceManager,
                        check_scope, default_max_bytes, detach, getWorkspaceManager, leverageTo, owner_of)

__all__ = ["AllocationPolicy", "LearningPolicy", "LocationPolicy", "MemoryWorkspace", "MirroringPolicy",
           "ND4JWorkspaceException", "ResetPolicy", "SpillPolicy", "WorkspaceConfiguration", "WorkspaceManager",
           "check_scope", "default_max_bytes", "detach", "getWorkspaceManager", "leverageTo", "owner_of"]
