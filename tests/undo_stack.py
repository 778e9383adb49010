"""UndoRedoStackManager as the reference's matrix tests use it (matrix/src/test/undoRedoStackManager.ts, a test-only
copy of framework/undo-redo): undo and redo stacks of operation stacks of IRevertibles.  Test infrastructure: the
IUndoConsumer the SharedMatrix undo provider (fluidframework_amd/undo.py) pushes to."""


class _Stack:
    """Stack over an array: push = unshift, pop = shift (undoRedoStackManager.ts:23-51)."""

    def __init__(self, *items):
        self.items = []
        for x in items:
            self.push(x)

    def empty(self):
        return not self.items

    def top(self):
        return self.items[0] if self.items else None

    def pop(self):
        return self.items.pop(0) if self.items else None

    def push(self, item):
        self.items.insert(0, item)


class _UndoRedoStack(_Stack):
    def close_current_operation_if_in_progress(self):  # :66-72
        if self.top() is not None:
            self.push(None)


class UndoRedoStackManager:
    NONE, REDO, UNDO = 0, 1, 2

    def __init__(self):
        self.undo_stack = _UndoRedoStack()
        self.redo_stack = _UndoRedoStack()
        self.mode = self.NONE

    @staticmethod
    def _revert(revert_stack, push_stack):  # :88-121
        push_stack.close_current_operation_if_in_progress()
        while not revert_stack.empty() and revert_stack.top() is None:
            revert_stack.pop()
        if not revert_stack.empty():
            op_stack = revert_stack.pop()
            if op_stack is not None:
                while not op_stack.empty():
                    op = op_stack.pop()
                    if op is not None:
                        op.revert()
        revert_stack.close_current_operation_if_in_progress()
        push_stack.close_current_operation_if_in_progress()

    def close_current_operation(self):
        if self.mode == self.NONE:
            self.undo_stack.close_current_operation_if_in_progress()

    def undo_operation(self):
        if self.undo_stack.empty():
            return False
        self.mode = self.UNDO
        self._revert(self.undo_stack, self.redo_stack)
        self.mode = self.NONE
        return True

    def redo_operation(self):
        if self.redo_stack.empty():
            return False
        self.mode = self.REDO
        self._revert(self.redo_stack, self.undo_stack)
        self.mode = self.NONE
        return True

    def push_to_current_operation(self, revertible):  # :158-184
        if self.mode == self.NONE:
            stack = self.undo_stack
            self._clear_redo_stack()
        elif self.mode == self.REDO:
            stack = self.undo_stack
        else:
            stack = self.redo_stack
        op_stack = stack.top()
        if op_stack is None:
            stack.push(_Stack(revertible))
        else:
            op_stack.push(revertible)

    def _clear_redo_stack(self):  # :186-198
        while not self.redo_stack.empty():
            op_stack = self.redo_stack.pop()
            if op_stack is not None:
                while not op_stack.empty():
                    op = op_stack.pop()
                    if op is not None:
                        op.discard()
